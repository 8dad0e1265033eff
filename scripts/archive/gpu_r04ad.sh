#!/bin/bash
# Final profile pass on the frozen round-4 sources: bench (trace + PMC -> pdhg_valu / pdhg_traffic) and the chain /
# ICE kernels (profile_kernels.sh).
set -o pipefail
bash scripts/profile_round.sh r04ad || exit 1
bash scripts/profile_kernels.sh r04ad || exit 1
