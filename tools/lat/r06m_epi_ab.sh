# r06m: the pair kernel's epilogue without its leading workgroup barrier (this build) against the
# same sources with it (tools/lat/libbase_r06.so), the C2 sweep in the driver's form, alternating,
# three rounds; the pair-kernel parity tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py tests/test_gpu_twophase.py -m gpu > $O/r06m_tests.txt 2>&1 && tail -1 $O/r06m_tests.txt &&
for r in 1 2 3; do
  for L in tools/lat/libbase_r06.so msccl_amd/libmsccl_amd.so; do
    MSCCL_AMD_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --pmc off --no-secondary \
      > $O/r06m_sw.json 2>> $O/r06m_sw.err || exit 1
    python -c "
import json; d = json.load(open('$O/r06m_sw.json'))
print('$(basename $L)', 'value %.1f avg %.2f |' % (d['value'], d['avg_busbw']), ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms'] * 1e3) for s in d['sweep']))" | tee -a $O/r06m_epi_ab.txt
  done
done
