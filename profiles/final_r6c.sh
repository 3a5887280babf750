# Round 6 final pass on the last tree (shipped library rebuilt after the tuning-only split-query
# variant): the whole GPU suite (margins.jsonl), smoke, config-3 and config-2 lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/margins.jsonl
bash profiles/gpu_session.sh r6h tests smoke cfg3 cfg2
