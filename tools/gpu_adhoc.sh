#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: the full GPU pass on the round's final tree
bash tools/gpu_full.sh r03f2
