#!/bin/bash
# Config 3 (DCM + PV annual 5-minute window, long team): option sweep.
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 300 python -u scripts/probe_config3_opts.py dcm '{}' '{"primal_weight_theta": 0.5}' '{"primal_weight_theta": 0.25}' \
  '{"primal_weight_theta": 0.75}' '{"check_every": 64}' '{"check_every": 16}' '{"restart_sufficient": 0.1, "restart_necessary": 0.9}' \
  '{"restart_sufficient": 0.3, "restart_necessary": 0.7}' '{"restart_artificial": 0.05}' '{"restart_artificial": 0.3}' \
  '{"ruiz_iters": 20}' '{"ruiz_iters": 4}' '{"reflection": 0.9}' > $O/opts.log 2>&1 || { echo "probe failed"; tail -20 $O/opts.log; exit 1; }
grep -v amdgpu.ids $O/opts.log
