export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_stream_check.sh r03o && TAG=r03o LIBS="ab/base.so product" bash tools/stream_ab.sh
