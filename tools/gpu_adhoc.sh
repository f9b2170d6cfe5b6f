export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python3 tools/txrx_overlap.py 1 2 4 8 16 1 4
