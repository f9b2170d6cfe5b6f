mkdir -p gpurun_out
for s in 5242880 10485760 20971520 41943040 167772160; do
  timeout -k 10 120 python tools/kbench.py --configs B --samples $s --reps 50 >> gpurun_out/kbench_sizes.jsonl 2>/dev/null || exit 1
done
