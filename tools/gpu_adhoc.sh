#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: the full GPU pass after the tx occupancy bound
bash tools/gpu_full.sh r03z
