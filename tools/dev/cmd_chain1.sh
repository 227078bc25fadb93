# one chain (no overlap): pure per-kernel durations per level from a kernel trace
set -u
export TMPDIR=/tmp
SVO_CHAINS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c1prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-secondary --core-only > gpurun_out/c1.log 2>&1 || exit $?
python3 - <<'PY'
import csv, re, collections, statistics
rows = list(csv.DictReader(open('gpurun_out/c1prof/run_kernel_trace.csv')))
def nm(k):
    m = re.search(r'(align_\w+)(<[^>(]*>)?', k); return (m.group(1) + (m.group(2) or '')) if m else None
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), nm(r['Kernel_Name']), r['Grid_Size_X']) for r in rows if nm(r['Kernel_Name']))
# the last 15 align dispatches = one chain step of 5 levels
d = collections.defaultdict(list)
for s, e, k, g in ev[-45:]:
    d[(k, g)].append((e - s) / 1e3)
for k, v in sorted(d.items()):
    print(k, [round(x, 1) for x in v])
PY
