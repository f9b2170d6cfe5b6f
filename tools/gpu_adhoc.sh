export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
bash tools/sq_stream.sh && grep "stream_decode\|stream_walk" gpurun_out/sq_stream.txt | grep "INSTS_VALU\|WAVES \|WAVE_CYCLES\|ACTIVE_INST_VALU\|BUSY_CYCLES"
