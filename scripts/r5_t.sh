set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/calltrace O=gpurun_out/calltrace bash scripts/trace_call.sh || exit 1
python3 - <<'PY'
import csv, glob, collections
kt = glob.glob("gpurun_out/calltrace/trace/**/*kernel_trace.csv", recursive=True)
at = glob.glob("gpurun_out/calltrace/trace/**/*hip_api_trace.csv", recursive=True)
for f in kt:
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in d.items(): print("kernel", k, len(v), "median us %.2f" % sorted(v)[len(v)//2])
for f in at:
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        d[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:12]: print("api", k, len(v), "median us %.2f" % sorted(v)[len(v)//2], "total %.0f" % sum(v))
PY
