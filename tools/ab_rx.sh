# A/B of two builds of the library on one box: kbench config B rx/tx, alternating
# (A = the in-tree library, B = $AB_LIB), $AB_ROUNDS rounds each.
export TMPDIR=/tmp
for r in $(seq ${AB_ROUNDS:-3}); do
  for v in A B; do
    if [ $v = A ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$AB_LIB; fi
    timeout -k 10 120 python tools/kbench.py --configs ${AB_CONFIGS:-B} --reps 30 2>/dev/null | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if d['variant'] in ('rx(constell+bytes+ber)', 'rx(bytes)', 'tx+awgn'): print('$v', d['config'], d['variant'], d['ms'])
" || exit 1
  done
done
