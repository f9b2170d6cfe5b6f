#!/bin/bash
# A/B/C... of library builds on one box: kbench per library, alternating,
# $AB_ROUNDS rounds.  AB_LIBS="base:path1 nofft:path2 ..." (base = in-tree lib
# when path is "-").  Output: one line per (round, lib, variant, ms).
export TMPDIR=/tmp
for r in $(seq ${AB_ROUNDS:-3}); do
  for spec in $AB_LIBS; do
    name=${spec%%:*}; path=${spec#*:}
    if [ "$path" = "-" ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$path; fi
    timeout -k 10 120 python tools/kbench.py --configs ${AB_CONFIGS:-B} --reps 30 2>/dev/null | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print('$r', '$name', d['config'], d['variant'], round(d['ms'], 4), round(d.get('GBps', 0)))
" || exit 1
  done
done
