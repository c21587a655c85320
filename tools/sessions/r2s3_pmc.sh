# Session-3 evidence, part 1: PMC passes of the dominant kernels (k_wave at C2,
# k_long at C3 -- the sizes bench.py runs) on the current tree.
set -u
export TMPDIR=/tmp
bash tools/pmc_session.sh ${TAG:-r2s3}_pmc_c2 c2 'k_wave' 1000000 || exit 1
bash tools/pmc_session.sh ${TAG:-r2s3}_pmc_c3 c3 'k_long' 100000 || exit 1
echo pmc done
