# HBM bytes per kernel (FETCH_SIZE / WRITE_SIZE passes, FETCH doubled per the gfx950 note) + kernel durations, one frame group of 160 frames: bash tools/hbm_per_kernel.sh
export TMPDIR=/tmp
O=gpurun_out/hbm27; mkdir -p $O
Q="python3 tools/quick_perf.py --frames 160 --per-launch 160 --count-frames 1"
RT_GROUPS=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- $Q > $O/f.log 2>&1 || { echo f failed; exit 1; }
RT_GROUPS=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- $Q > $O/w.log 2>&1 || { echo w failed; exit 1; }
RT_GROUPS=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- $Q > $O/t.log 2>&1 || { echo t failed; exit 1; }
python3 - <<'PY'
import csv, glob, collections
O='gpurun_out/hbm27'
def load(d, cname):
    rows=[]
    for f in glob.glob(O+'/'+d+'/*counter_collection.csv'):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name']==cname: rows.append((int(r['Dispatch_Id']), r['Kernel_Name'].split('(')[0][-28:], float(r['Counter_Value'])))
    return sorted(rows)
fe=load('f','FETCH_SIZE'); wr=load('w','WRITE_SIZE')
kt=[r for r in csv.DictReader(open(glob.glob(O+'/t/*kernel_trace.csv')[0]))]
dur=[(int(r['Dispatch_Id']), r['Kernel_Name'].split('(')[0][-28:], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6) for r in kt]
dur=sorted(dur)
# align by order among wf_ kernels of the timed 160-frame launch (the largest camera trace marks it)
def wf(rows): return [r for r in rows if 'wf_' in r[1]]
fe, wr, du = wf(fe), wf(wr), wf(dur)
n=min(len(fe),len(wr),len(du))
print('n', len(fe), len(wr), len(du))
for i in range(n):
    if du[i][2] > 0.5:
        f=fe[i][2]*2*1024/1e9; w=wr[i][2]*1024/1e9  # FETCH_SIZE kB x2 (gfx950 per guide), WRITE kB
        print(f"{du[i][1]:28s} {du[i][2]:7.2f} ms  fetch {f:7.2f} GB  write {w:6.2f} GB  -> {(f+w)/du[i][2]:6.2f} TB/s")
PY
