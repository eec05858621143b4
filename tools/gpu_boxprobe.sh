#!/bin/bash
# Box probe (round 5): VRAM use and clocks before our work, the two-column
# stream rate, then two PMC passes over the C3 bench (translation and fabric
# counters; k_sieve_l1 time from the same processes) -> $OUT/probe.txt
# Usage: bash tools/gpu_boxprobe.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-gpurun_out/probe}
mkdir -p $OUT
rocm-smi --showmemuse --showmeminfo vram > $OUT/smi.txt 2>&1 || true
[ -x tools/stream_bench ] && { timeout -k 10 120 tools/stream_bench > $OUT/stream.txt 2>&1 || true; }
BENCH="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-api"
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum"
P2="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_LEVEL_sum"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc$i -o run --output-format csv -- $BENCH > $OUT/pmc$i.log 2>&1 || { echo "probe PMC pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 - $OUT <<'PY' > $OUT/probe.txt
import csv, glob, json, sys, collections
out = sys.argv[1]
print(open(out + "/smi.txt").read().strip().splitlines()[-6:])
try:
    print([l for l in open(out + "/stream.txt") if "tiles2 Q=4" in l])
except OSError:
    pass
for i in (1, 2):
    line = [l for l in open(f"{out}/pmc{i}.log") if l.startswith("{")]
    r = json.loads(line[-1]) if line else {}
    print(f"pass {i}: bench k_sieve_l1 ms", round(r.get("kernels", {}).get("k_sieve_l1", {}).get("ms", -1), 3))
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/pmc{i}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_sieve_l1" in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"  {k}: mean {sum(v) / len(v):.4g} over {len(v)} launches")
PY
cat $OUT/probe.txt
