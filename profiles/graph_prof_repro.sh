# rocprofv3 --kernel-trace of hipGraph replays (whisper.coreml_amd/tools/graph_prof_repro):
# which of node count, replay count and argument size triggers the segfault
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "400 64 20" "4000 64 2" "400 64 200" "2000 64 2" "1000 64 8" "8000 64 1" "100 64 800"; do
  set -- $cfg
  timeout -k 10 60 rocprofv3 --kernel-trace -d gpurun_out/repro_$1_$3 -o run -- ./whisper.coreml_amd/tools/graph_prof_repro $1 $2 $3 > gpurun_out/repro_$1_$3.log 2>&1
  echo "nodes $1 argb $2 reps $3 dispatches $(( $1 * $3 )) rc=$?"
done
