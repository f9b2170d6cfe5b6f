# Scratch slot for one-off GPU commands (`gpurun -- bash tools/gpu_adhoc.sh`);
# its content changes with the experiment at hand and is not part of any flow.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python3 tools/ab_step.py
