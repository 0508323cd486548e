#!/bin/bash
# Profile one workload: kernel trace + stats, then separate --pmc passes (HBM bytes, SQ instruction mix, LDS waits).
# Big raw CSVs are summarised on the box and removed (gpurun copies back at most 64 MiB).
# Usage (via gpurun): bash scripts/gpu_prof.sh TAG [bench args...]     e.g. gpu_prof.sh p_c2 --steps 2 --warmup 1
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BA="--no-cpu-baseline --no-parity --no-e2e --no-c3 --window-markers $@"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/kt -o run --output-format csv -- python3 $R/bench.py $BA > $R/$OUT/kt.log 2>&1 || { echo kt failed; tail -3 $R/$OUT/kt.log; exit 1; }
tail -1 $R/$OUT/kt.log | cut -c1-300
STATS=$(find $R/$OUT/kt -name "*kernel_stats.csv" | head -1)
cp $STATS $R/$OUT/kernel_stats.csv
# per-kernel averages over the timed steps only: the kernels that start between the bench's two window markers
# (bench.py --window-markers: a spin_kernel right before the first timed step and right after the closing sync), so
# neither the warm-up steps nor set-up launches (fills, creation) are charged to a step
TRACE=$(find $R/$OUT/kt -name "*kernel_trace.csv" | head -1)
python3 - "$TRACE" "$@" > $R/$OUT/kt_timed.txt <<'PY'
import csv, sys, collections
trace, args = sys.argv[1], sys.argv[2:]
def arg(name, dflt):
    return int(args[args.index(name) + 1]) if name in args else dflt
steps = arg("--steps", 1)
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(trace))]
marks = sorted(s for s, e, n in rows if "spin_kernel" in n)
assert len(marks) >= 2, "no timed-window markers in the trace (bench.py --window-markers)"
w0, w1 = marks[0], marks[-1]
ev = collections.defaultdict(list)
for s, e, n in rows:
    if w0 < s < w1 and "spin_kernel" not in n:
        n = n.split("(")[0].replace("void ", "").replace("cc::", "")
        ev[n].append(e - s)
tot = sum(sum(v) for v in ev.values())
print(f"timed window {(w1 - w0) / 1e6:.3f} ms over {steps} steps ({(w1 - w0) / 1e6 / steps:.3f} ms/step between the "
      f"markers); kernels in it {tot / 1e6 / steps:.3f} ms/step")
print(f"{'kernel':44s} {'calls':>6s} {'avg_us':>10s} {'ms/step':>10s}")
for n, v in sorted(ev.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n[:44]:44s} {len(v):6d} {sum(v) / len(v) / 1e3:10.1f} {sum(v) / steps / 1e6:10.3f}")
PY
# idle gaps of the timed steps: the union of all kernels' intervals between the window markers, and the
# largest gaps with the kernels on either side (host round trips show up here)
python3 - "$TRACE" "$@" > $R/$OUT/kt_gaps.txt <<'PY'
import csv, sys
trace, args = sys.argv[1], sys.argv[2:]
def arg(name, dflt):
    return int(args[args.index(name) + 1]) if name in args else dflt
steps, warm = arg("--steps", 1), arg("--warmup", 1)
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cc::", "")[:40])
            for r in csv.DictReader(open(trace)))
if not ev:
    sys.exit()
marks = [e[0] for e in ev if "spin_kernel" in e[2]]
ev = [e for e in ev if marks[0] < e[0] < marks[-1] and "spin_kernel" not in e[2]] if len(marks) >= 2 else ev
busy, gaps = 0, []
cs, ce, last = ev[0][0], ev[0][1], ev[0][2]
for s, e, n in ev[1:]:
    if s > ce:  # an idle gap before this kernel
        busy += ce - cs
        gaps.append((s - ce, last, n))
        cs, ce, last = s, e, n
    elif e > ce:
        ce, last = e, n
busy += ce - cs
cur_end = ce
span = cur_end - ev[0][0]
print(f"timed window {span / 1e6:.3f} ms, kernels busy (union) {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms "
      f"in {len(gaps)} gaps ({sum(g[0] for g in gaps if g[0] > 10000) / 1e6:.3f} ms in gaps > 10 us)")
for g in sorted(gaps, reverse=True)[:25]:
    print(f"  {g[0] / 1e3:9.1f} us  after {g[1]:40s} before {g[2]}")
PY
find $R/$OUT/kt -name "*kernel_trace.csv" -delete
i=0
[ -n "$KT_ONLY" ] && PMCS="" || PMCS=1
for CNT in ${PMCS:+ "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY"}; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CNT -d $R/$OUT/pmc$i -o run --output-format csv -- python3 $R/bench.py $BA > $R/$OUT/pmc$i.log 2>&1 || { echo "pmc $i ($CNT) failed"; tail -3 $R/$OUT/pmc$i.log; }
  (cd $R && python3 scripts/pmc_kernel_summary.py $OUT/pmc$i > $OUT/pmc${i}_summary.txt 2>&1)
  find $R/$OUT/pmc$i -name "*.csv" -delete
done
cd $R
python3 -c "
import csv
rows = list(csv.DictReader(open('$OUT/kernel_stats.csv')))
print(f\"{'kernel':44s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>10s}\")
for r in rows:
    n = r['Name'].split('(')[0].replace('void ', '').replace('cc::', '')
    print(f\"{n[:44]:44s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.1f} {float(r['TotalDurationNs'])/1e6:10.3f}\")
" > $OUT/kt_summary.txt
head -25 $OUT/kt_summary.txt
head -12 $OUT/kt_timed.txt
du -sh $OUT
echo done
