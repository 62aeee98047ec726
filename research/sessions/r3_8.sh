# N=1 fp8 / tp_rowwise benches (JSON kept) and the runner's --pmc end to end (rocpd databases
# kept off gpurun_out: only the CSV with the per-kernel counter means comes back)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_8
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.log 2>&1 || { tail -20 $O/bench_fp8.log; exit 1; }
grep -a metric $O/bench_fp8.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > $O/bench_row.log 2>&1 || { tail -20 $O/bench_row.log; exit 1; }
grep -a metric $O/bench_row.log | cut -c1-200
timeout -k 10 300 python -m ddlb_amd --primitive tp_columnwise -m 65536 -n 1024 -k 1024 --dtype bfloat16 --impl "native" --impl "compute_only;size=unsharded;gemm=torch_nt" --num-iterations 20 --num-warmups 3 --pmc default --pmc-dir /tmp/ddlb_pmc --output-csv $O/cli_pmc.csv > $O/cli_pmc.log 2>&1 || { tail -30 $O/cli_pmc.log; exit 1; }
du -sh /tmp/ddlb_pmc; python -c "
import csv, json
for r in csv.DictReader(open('$O/cli_pmc.csv')):
    print(r['implementation'][:60], r['mean_time (ms)'], r['valid'])
    for k, v in json.loads(r['pmc']).items(): print('   ', k[:70], {c: round(x) for c, x in v.items()})
"
