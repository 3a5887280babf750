# Round 6 final pass, part B: config-5 and config-4 (N = 1) lines, graph-mode step profiles (20
# windows, one window, turbo), the eager rocprofv3 kernel trace of the bench, PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash profiles/gpu_session.sh r6f cfg5 cfg4 step20 step1 stepturbo profeager pmc
