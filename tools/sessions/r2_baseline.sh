#!/bin/bash
# Round-2 baseline counters on the round-1 kernels: k_long at C3, k_wave at C2.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/pmc_session.sh" r2a_c3_long c3 'k_long' && \
bash "$R/tools/pmc_session.sh" r2a_c2_wave c2 'k_wave'
