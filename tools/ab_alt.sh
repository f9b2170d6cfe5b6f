#!/bin/bash
# A/B of library builds on the bench's tx -> rx pair (kbench --alt), alternating.
# AB_LIBS="name:path ..." (path "-" = in-tree library), AB_ROUNDS rounds.
export TMPDIR=/tmp
for r in $(seq ${AB_ROUNDS:-3}); do
  for spec in $AB_LIBS; do
    name=${spec%%:*}; path=${spec#*:}
    if [ "$path" = "-" ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$path; fi
    timeout -k 10 120 python tools/kbench.py --configs ${AB_CONFIGS:-B} --reps 30 --alt 2>/dev/null | grep '"alt' | sed "s/^/$r $name /" || exit 1
  done
done
