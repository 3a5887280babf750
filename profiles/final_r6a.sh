# Round 6 final pass, part A: the whole GPU suite (margins.jsonl), smoke, config-3 line (with the
# CPU baseline) and config-2 line, on the final tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/margins.jsonl
bash profiles/gpu_session.sh r6f tests smoke cfg3 cfg2
