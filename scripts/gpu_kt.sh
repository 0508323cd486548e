#!/bin/bash
# Kernel trace + stats of one bench configuration (no counters).  Usage: bash scripts/gpu_kt.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-parity --no-e2e "$@" > $R/$OUT/kt.log 2>&1 || { echo kt failed; tail -3 $R/$OUT/kt.log; exit 1; }
cd $R
STATS=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
cp $STATS $OUT/kernel_stats.csv
TRACE=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 - "$TRACE" > $OUT/gaps.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
gaps = {}
for a, b in zip(rows, rows[1:]):
    g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
    key = (a["Kernel_Name"].split("(")[0][-40:], b["Kernel_Name"].split("(")[0][-40:])
    gaps.setdefault(key, []).append(g)
print(f"kernels {len(rows)} busy {busy/1e6:.3f} ms span {span/1e6:.3f} ms")
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:15]:
    print(f"{sum(v)/1e6:8.3f} ms over {len(v):5d} gaps (avg {sum(v)/len(v)/1e3:7.1f} us)  {k[0]} -> {k[1]}")
PY
find $OUT/kt -name "*kernel_trace.csv" -delete
python3 -c "
import csv
rows = list(csv.DictReader(open('$OUT/kernel_stats.csv')))
for r in rows[:25]:
    n = r['Name'].split('(')[0].replace('void ', '').replace('cc::', '')
    print(f\"{n[:44]:44s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.1f} {float(r['TotalDurationNs'])/1e6:10.3f}\")
" > $OUT/kt_summary.txt
cat $OUT/kt_summary.txt; cat $OUT/gaps.txt
