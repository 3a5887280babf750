# Round 5 final GPU pass: GPU suite, smoke, config 3 / config 2 bench lines, PMC traffic
set -o pipefail
T=${1:-r5l}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$T.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.txt 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > gpurun_out/cfg3_$T.json 2> gpurun_out/cfg3_$T.err || exit 3
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 > gpurun_out/cfg2_$T.json 2> gpurun_out/cfg2_$T.err || exit 4
bash profiles/pmc_pass.sh || exit 5
