export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
bash tools/sq_stream.sh && grep stream_decode gpurun_out/sq_stream.txt
