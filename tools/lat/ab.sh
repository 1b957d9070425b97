set -o pipefail
run() { MSCCL_AMD_LIB=$1 timeout -k 5 60 python3 tools/lat_one.py --iters 300 --graph --schedule pair --bytes $2 --ranks 2 --instances 16 2>&1 | grep -v amdgpu.ids | sed "s|^|$1 |"; }
run tools/lat/libvar_pf4.so 8192 || exit 1
for rep in 1 2; do for L in tools/lat/libvar_base.so tools/lat/libvar_pf4.so tools/lat/libvar_pf1.so; do for b in 8192 65536 1048576 4194304 33554432; do run $L $b || exit 1; done; done; done
MSCCL_AMD_LIB=tools/lat/libvar_pf4.so timeout -k 10 200 python3 bench.py --no-cpu --pmc off --no-secondary > gpurun_out/r05l_pf_bench.json 2> gpurun_out/r05l_pf_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r05l_pf_bench.json')); print('pf4 bench', d['value'], d['avg_busbw'], d['verified'], [s['bytes'] for s in d['sweep'] if not s['verified']])"
