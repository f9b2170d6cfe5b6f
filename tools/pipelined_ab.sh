#!/bin/bash
# Same-box A/B of the two-context ("pipelined") stream receive against serial
# calls, across the round-3 window in which the pipelined figure fell below
# serial: cce3421 (before f93d7a8), f93d7a8 (decode 126 -> 120 VGPRs) and the
# current tree. Each tree runs its own tools/stream_bench.py against its own
# library (ab/<commit>: git worktrees built in this container). Two rounds,
# interleaved, so box drift shows.
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/${1:-r04}_pipelined_ab.jsonl
: > $OUT
for round in 1 2; do
  for tree in ab/cce3421 ab/f93d7a8 .; do
    for fmt in "" "--i16"; do
      for p in 1 2; do
        r=$(cd $tree && timeout -k 10 120 python tools/stream_bench.py --frames 16384 --reps 10 --pipeline $p $fmt 2>/dev/null) || { echo "failed: $tree $fmt $p"; exit 1; }
        echo "{\"tree\": \"$tree\", \"round\": $round, \"fmt\": \"${fmt:-f64}\", \"result\": $r}" >> $OUT
      done
    done
  done
done
python3 - "$OUT" <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for r in rows:
    d = r["result"]
    print(r["round"], r["tree"], r["fmt"], "pipeline", d["pipeline"], "ms", d["ms"], "G/s", d["G_stream_samples_per_s"])
EOF
