#!/bin/bash
# PMC HBM-traffic passes (one counter group per run, kernel trace only): writes
# gpurun_out/traffic.json; copy it to profiles/<round>/traffic.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_f -o run --output-format csv -- \
  python3 $R/profiles/pmc_traffic.py run > $R/gpurun_out/pmc_f.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_w -o run --output-format csv -- \
  python3 $R/profiles/pmc_traffic.py run > $R/gpurun_out/pmc_w.log 2>&1 || exit 2
cd $R && python3 profiles/pmc_traffic.py parse gpurun_out/pmc_f gpurun_out/pmc_w > gpurun_out/traffic.json
