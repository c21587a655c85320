# PMC passes of k_wave at C2 only (after a k_wave-only change).
set -u
export TMPDIR=/tmp
bash tools/pmc_session.sh ${TAG:-r2s3}_pmc_c2 c2 'k_wave' 1000000 || exit 1
echo pmc done
