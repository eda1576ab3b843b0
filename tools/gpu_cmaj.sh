# chunk-major K order A/B on the heads (run on the GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 300 ./tools/convbench 20 head > gpurun_out/cb_heads.txt 2>&1 || { echo "convbench failed"; tail gpurun_out/cb_heads.txt; exit 1; }
cat gpurun_out/cb_heads.txt
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/cb_pmc -o run -- ./tools/convbench 3 "head L" > gpurun_out/cb_pmc.log 2>&1 || { echo "pmc failed"; tail gpurun_out/cb_pmc.log; exit 1; }
python3 - <<'P'
import csv,glob,collections
f=glob.glob('gpurun_out/cb_pmc/**/*counter_collection.csv',recursive=True)
print(f)
agg=collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    agg[(r['Kernel_Name'][:60], r['Grid_Size'] if 'Grid_Size' in r else r.get('Grid_Size_X',''))].append(float(r['Counter_Value']))
for k,v in agg.items(): print(k, len(v), 'FETCH_SIZE KiB avg %.0f'%(sum(v)/len(v)))
P
