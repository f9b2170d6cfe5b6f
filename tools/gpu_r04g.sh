#!/bin/bash
# round-4 experiments (trees under ab/, built in this container, not committed):
#  1. the two halves of f93d7a8 (decode gains / sync-stage changes) in the
#     pipelined A/B against cce3421 and f93d7a8;
#  2. the wide decode's stages alone: sync stage only (exp_sync) and rx stage
#     only (exp_rx), kernel trace of the config-B stream.
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04g}
OUT=gpurun_out/${TAG}_pipelined_split.jsonl
: > $OUT
for round in 1 2; do
  for tree in ab/cce3421 ab/split_gains ab/split_sync ab/f93d7a8; do
    for p in 1 2; do
      r=$(cd $tree && timeout -k 10 120 python tools/stream_bench.py --frames 16384 --reps 10 --pipeline $p --i16 2>/dev/null) || { echo "failed: $tree $p"; exit 1; }
      echo "{\"tree\": \"$tree\", \"round\": $round, \"fmt\": \"i16\", \"result\": $r}" >> $OUT
    done
  done
done
python3 - "$OUT" <<'EOF'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l); d = r["result"]
    print(r["round"], r["tree"], "contexts", d["pipeline"], "ms", d["ms"], "G/s", d["G_stream_samples_per_s"])
EOF
for tree in ab/exp_sync ab/exp_rx .; do
  n=$(basename $tree); [ "$n" = "." ] && n=head
  (cd $tree && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_wide_$n -o run -- python3 tools/stream_bench.py --config B --frames 4096 --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_wide_$n.json 2>/dev/null) || { echo "prof failed $tree"; exit 1; }
  f=$(find gpurun_out/${TAG}_wide_$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; grep -E "stream_decode_wide|stream_walk" "$f" | cut -d, -f1-6
done
