#!/bin/bash
# HBM traffic of the config-4 stream kernels: separate rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE) over tools/stream_bench.py, summarised per kernel
# (mean over its dispatches) into gpurun_out/pmc_stream${SUF}.json; extra
# arguments go to stream_bench.py (e.g. SUF=_i16 tools/pmc_stream.sh --i16).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcs_fetch$SUF -o run -- python3 tools/stream_bench.py --reps 1 "$@" > $R/gpurun_out/pmcs_fetch$SUF.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcs_write$SUF -o run -- python3 tools/stream_bench.py --reps 1 "$@" > $R/gpurun_out/pmcs_write$SUF.log 2>&1 && \
SUF=$SUF python3 - <<'PY' > $R/gpurun_out/pmc_stream$SUF.json
import csv, glob, json, collections, os
suf = os.environ.get("SUF", "")
acc = collections.defaultdict(list)
for ctr, path in (("FETCH_SIZE", f"gpurun_out/pmcs_fetch{suf}/run_counter_collection.csv"),
                  ("WRITE_SIZE", f"gpurun_out/pmcs_write{suf}/run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        for key in ("stream_walk_kernel", "stream_decode_wide_kernel", "compact_kernel", "resolve_kernel", "cfo_kernel", "stream_params_kernel", "stream_sync_kernel",
                    "rx_stream2_kernel", "stream_decode_kernel", "rx_kernel"):
            if key in k and r["Counter_Name"] == ctr:
                acc[(key, ctr)].append(float(r["Counter_Value"]))
out = {"note": "KiB per dispatch (mean over the bench's dispatches: warm-up + 1 timed); "
               "FETCH_SIZE under-reports wide streaming reads 2x on gfx950 (MI355X_MICROARCH.md), "
               "so reads lie between 1x and 2x FETCH_SIZE for these mixed access patterns"}
for (key, ctr), v in sorted(acc.items()):
    out.setdefault(key, {})[ctr + "_kib"] = sum(v) / len(v)
print(json.dumps(out, indent=1))
PY
