# Scratch slot for one-off GPU commands (`gpurun -- bash tools/gpu_adhoc.sh`);
# its content changes with the experiment at hand and is not part of any flow.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/gpu_stream_check.sh r03r && TAG=r03r LIBS="ab/base.so product" bash tools/stream_ab.sh
