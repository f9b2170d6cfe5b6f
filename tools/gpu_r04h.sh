#!/bin/bash
# round-4 experiments (trees under ab/, built in this container, not committed):
#  1. pipelined A/B: which hunk of f93d7a8's sync-stage change removes the
#     two-context overlap (each reverted alone on HEAD, and all three);
#  2. the wide decode with the second workgroup of each CU started late
#     (convoy test: do the two frames of a CU run their stages in phase?).
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04h}
OUT=gpurun_out/${TAG}_pipelined_rev.jsonl
: > $OUT
for round in 1 2; do
  for tree in ab/cce3421 . ab/rev_all ab/rev_h1 ab/rev_h2 ab/rev_h3; do
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
for tree in . ab/stag10 ab/stag25 ab/stag40; do
  n=$(basename $tree); [ "$n" = "." ] && n=head
  (cd $tree && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_wide_$n -o run -- python3 tools/stream_bench.py --config B --frames 4096 --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_wide_$n.json 2>/dev/null) || { echo "prof failed $tree"; exit 1; }
  f=$(find gpurun_out/${TAG}_wide_$n -name "*kernel_stats.csv" | head -1)
  echo "== $n $(python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_wide_$n.json'));print(d['ms'], d['frames_error_free'])")"; grep -E "stream_decode_wide" "$f" | cut -d, -f1-4
done
