#!/bin/bash
# One GPU session, run from the repo root on the GPU box: the steps named in STEPS, outputs under
# gpurun_out/$TAG_*.  Every GPU step runs under its own time limit and the first failure ends the
# session (nothing more touches the GPU after a fault, an abort or a time limit).
#   suite     the GPU test suite (pytest -m gpu)
#   lat       graph-replay latency per launch (tools/lat_one.py) of every library in LIBS on the
#             2-rank pair tier, the 8-rank C3 small tier and the flat fold, same box
#   trace     tools/lat_trace.py on LATLIB (a MSCCL_LAT_TRACE build, see msccl_amd/csrc/Makefile)
#   bench     the default bench line (N=1, C2, live PMC)
#   c345      the 8-rank C3 shape plus C4 / C5 (co-resident ranks)
#   spawn     the 2-process launcher rehearsal on one GPU and the launcher's refusal
#   sweep     bench.py sweeps of every library in LIBS (C2 2 ranks, then C3 shape 8 ranks fp16)
#   xover     the lowered fold against the interpreter, 8 KiB - 128 KiB (MSCCL_AMD_LOWER_MAX_BYTES)
#   c4trace   where the 8-rank C4 ring launch waits (tools/trace_report.py --summary)
#   c4knobs   the 8-rank C4 shape under each environment of C4ENVS (';'-separated)
#   c3inst    the 8-rank C3 shape at 32 MiB for each all-pairs instance count in C3INST, and its trace
#   xcdpmc    rocprofv3's counter list and per-instance TCC request counters of the C2 launch
#   prof      tools/profile.sh on the C2 headline (kernel stats, FETCH_SIZE, WRITE_SIZE)
#   prof8     the same on the 8-rank C3 shape and C4 / C5 (per-kernel traffic)
# e.g. STEPS="suite lat" LIBS="tools/ab/a.so msccl_amd/libmsccl_amd.so" TAG=r04a bash tools/gpu_session.sh
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r04}
STEPS=${STEPS:-"suite bench"}
LIBS=${LIBS:-msccl_amd/libmsccl_amd.so}
O=gpurun_out/$TAG
mkdir -p gpurun_out
fail() { echo "FAILED: $*"; [ -n "$2" ] && tail -30 "$2"; exit 1; }
lat() { timeout -k 5 90 python3 tools/lat_one.py --iters 300 --graph "$@" 2>&1 | grep -v amdgpu.ids; }
for step in $STEPS; do
  case $step in
  suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu ${SUITEARGS:--x} -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      > ${O}_suite.txt 2>&1 || fail suite ${O}_suite.txt
    tail -2 ${O}_suite.txt ;;
  lat)
    # LATSPECS: "schedule bytes ranks instances dtype [coll]" entries separated by ';'; LATENV: extra
    # environment for every run (e.g. MSCCL_AMD_LOWER=0)
    SPECS=${LATSPECS:-"pair 128 2 1 7;pair 4096 2 16 7;pair 65536 2 16 7;oneshot 128 8 4 6;oneshot 4096 8 4 6;fbtree 128 2 1 7;fbtree 128 8 1 6"}
    for L in $LIBS; do
      IFS=';' read -ra SP <<< "$SPECS"
      for spec in "${SP[@]}"; do
        set -- $spec
        r=$(env $LATENV MSCCL_AMD_LIB=$L timeout -k 5 90 python3 tools/lat_one.py --iters 300 --graph --schedule $1 \
            --bytes $2 --ranks $3 --instances $4 --dtype $5 --coll ${6:-ar} 2>&1 | grep -v amdgpu.ids) || fail "lat $L $spec"
        echo "$(basename $L) $LATENV $r" | tee -a ${O}_lat.txt
      done
    done ;;
  xover)
    # the fold (lowered) against the interpreter around MSCCL_AMD_LOWER_MAX_BYTES
    for spec in "pair 2 16 7" "oneshot 8 4 6" "allpairs 8 1 6"; do
      set -- $spec
      for b in 8192 16384 32768 65536 131072; do
        f=$(MSCCL_AMD_LOWER_MAX_BYTES=1073741824 lat --schedule $1 --bytes $b --ranks $2 --instances $3 --dtype $4) || fail "xover $spec $b"
        i=$(MSCCL_AMD_LOWER=0 lat --schedule $1 --bytes $b --ranks $2 --instances $3 --dtype $4) || fail "xover $spec $b"
        echo "fold: $f" | tee -a ${O}_xover.txt
        echo "interp: $i" | tee -a ${O}_xover.txt
      done
    done ;;
  c4trace)
    MSCCL_AMD_TRACE=1 timeout -k 10 300 python3 tools/trace_report.py --schedule ring --ranks 8 --instances 32 --proto Simple \
      --dtype 9 --bytes 268435456 --iters 3 --summary > ${O}_c4trace.txt 2>&1 || fail c4trace ${O}_c4trace.txt
    cat ${O}_c4trace.txt ;;
  c3inst)
    for i in ${C3INST:-2 4 8}; do
      env $C3ENV timeout -k 10 300 python3 bench.py --vranks 8 --dtype fp16 --sizes 33554432 --instances $i --no-cpu --pmc off \
        --no-secondary > ${O}_c3i.json 2>> ${O}_c3i.err || fail "c3inst $i" ${O}_c3i.err
      python3 -c "
import json; d = json.load(open('${O}_c3i.json')); s = d['sweep'][-1]
print('C3 32 MiB instances $i $C3ENV', s['kernel_ms'], s['busbw'], s['kernel'])" | tee -a ${O}_c3inst.txt
    done
    MSCCL_AMD_TRACE=1 timeout -k 10 300 python3 tools/trace_report.py --schedule allpairs --ranks 8 --instances 4 --proto LL \
      --dtype 6 --bytes 33554432 --iters 3 --summary > ${O}_c3trace.txt 2>&1 || fail c3trace ${O}_c3trace.txt
    cat ${O}_c3trace.txt ;;
  c4knobs)
    IFS=';' read -ra EV <<< "${C4ENVS:-NCCL_BUFFSIZE=4194304}"
    for e in "${EV[@]}"; do
      env $e timeout -k 10 300 python3 bench.py --vranks ${C4RANKS:-8} --dtype fp16 --sizes 128 --extras ${C4CFG:-C4} --no-cpu \
        --pmc off --no-secondary --steps 5 --warmup 2 > ${O}_c4k.json 2>> ${O}_c4k.err || fail "c4knobs $e" ${O}_c4k.err
      python3 -c "
import json
for c, d in json.load(open('${O}_c4k.json'))['configs'].items():
    print('${C4RANKS:-8} ranks', c, '$e', ' '.join('%s %s ms %s' % (k, v['kernel_ms'], v['memside_frac']) for k, v in d.items()
          if isinstance(v, dict) and 'kernel_ms' in v), d.get('verified'), d.get('error', ''))" | tee -a ${O}_c4knobs.txt
    done ;;
  xcdpmc)
    # per-XCD TCC counters of the C2 headline launch (JSON keeps every TCC instance x XCC value):
    # requests, read latency (RDREQ_LEVEL / RDREQ), DRAM credit stalls, hits / misses per XCD
    timeout -s KILL 60 rocprofv3 -L > ${O}_counters.txt 2>&1 || fail "rocprofv3 -L" ${O}_counters.txt
    for c in ${XCDCOUNTERS:-TCC_EA0_RDREQ TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_HIT TCC_MISS}; do
      d=gpurun_out/${TAG}_xcd_$c
      timeout -s KILL 120 rocprofv3 --pmc $c --output-format json -d $d -o run -- \
        python3 bench.py --sizes 33554432 --steps 10 --warmup 3 --no-cpu --quiet --no-secondary --pmc off --extras "" --eager \
        > /dev/null 2> ${O}_xcd_$c.err || fail "xcdpmc $c" ${O}_xcd_$c.err
      python3 tools/xcd_pmc.py $(find $d -name "*results.json" | head -1) > ${O}_xcd_$c.txt 2>&1 || fail "xcd_pmc $c" ${O}_xcd_$c.txt
      cat ${O}_xcd_$c.txt
      rm -rf $d
    done ;;
  prof)
    # rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes of the C2 headline
    # (tools/profile.sh -> gpurun_out/prof_${TAG}_final/, profiles/ files copied there)
    bash tools/profile.sh ${TAG}_final > ${O}_prof.txt 2>&1 || fail prof ${O}_prof.txt
    tail -c 600 ${O}_prof.txt ;;
  prof8)
    # the same passes over the 8-rank C3 shape (32 MiB) and the C4 / C5 configs: per-kernel traffic
    bash tools/profile.sh ${TAG}_extras8 --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu --quiet \
      --pmc off --no-secondary --steps 5 --warmup 2 > ${O}_prof8.txt 2>&1 || fail prof8 ${O}_prof8.txt
    tail -c 600 ${O}_prof8.txt ;;
  trace)
    MSCCL_AMD_LIB=${LATLIB:-tools/ab/libmsccl_amd_lat.so} MSCCL_AMD_TRACE=2 timeout -k 5 90 python3 tools/lat_trace.py \
      > ${O}_trace.txt 2>&1 || fail trace ${O}_trace.txt
    cat ${O}_trace.txt ;;
  bench)
    timeout -k 10 400 python3 bench.py > ${O}_bench.json 2> ${O}_bench.err || fail bench ${O}_bench.err
    python3 -c "import json; d=json.load(open('${O}_bench.json')); print('bench', d['value'], d['avg_busbw'], d['roofline']['frac'], d['roofline'].get('traffic_over_algorithmic'))" ;;
  c345)
    timeout -k 10 400 python3 bench.py --vranks 8 --dtype fp16 --sizes 128,65536,33554432 --extras C4,C5 --no-cpu --pmc off \
      --no-secondary > ${O}_c345_8.json 2> ${O}_c345_8.err || fail c345 ${O}_c345_8.err ;;
  spawn)
    MSCCL_AMD_BENCH_ONE_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --no-cpu --pmc off \
      > ${O}_spawn2.json 2> ${O}_spawn2.err || fail spawn ${O}_spawn2.err
    timeout -k 10 120 python3 bench.py --gpus 2 > ${O}_refuse2.json 2> ${O}_refuse2.err
    echo "refuse rc=$?" | tee ${O}_refuse2.rc ;;
  rehearse)
    # the driver's multi-GPU bench command, its N rank processes on cuda:0 (REHEARSE_N, default 8;
    # at 8 the C4 / C5 extras run too), the default K / W
    RN=${REHEARSE_N:-8}
    MSCCL_AMD_BENCH_ONE_GPU=1 timeout -k 10 600 python3 bench.py --gpus $RN ${REHEARSE_ARGS} \
      > ${O}_rehearse_$RN.json 2> ${O}_rehearse_$RN.err || fail "rehearse $RN" ${O}_rehearse_$RN.err
    python3 -c "
import json; d = json.load(open('${O}_rehearse_$RN.json'))
print('rehearse $RN', d['value'], d['avg_busbw'], d['verified'], {k: {p: v[p].get('kernel_ms') if isinstance(v.get(p), dict) else v.get(p) for p in v if p in ('allreduce', 'reduce_scatter', 'all_gather', 'verified', 'error')} for k, v in d.get('configs', {}).items()})" ;;
  traces)
    # per-transfer attribution (tools/trace_report.py --summary) of each "schedule ranks instances
    # proto dtype bytes" in TRSPECS (';'-separated)
    IFS=';' read -ra TS <<< "${TRSPECS:-allgather 8 8 Simple 7 67108864}"
    for spec in "${TS[@]}"; do
      set -- $spec
      MSCCL_AMD_TRACE=1 timeout -k 10 300 python3 tools/trace_report.py --schedule $1 --ranks $2 --instances $3 \
        --proto $4 --dtype $5 --bytes $6 --iters 3 ${TRMODE:---summary} >> ${O}_traces.txt 2>&1 || fail "traces $spec" ${O}_traces.txt
    done
    cat ${O}_traces.txt ;;
  envsweep)
    # the C2 sweep (or BARGS' shape) under each environment of SWEEPENVS (';'-separated, "-" = none)
    IFS=';' read -ra EV <<< "${SWEEPENVS:--}"
    for e in "${EV[@]}"; do
      [ "$e" = "-" ] && e=""
      env $e timeout -k 10 300 python3 bench.py --no-cpu --pmc off ${ES_SEC:---no-secondary} ${BARGS} > ${O}_es.json 2>> ${O}_es.err \
        || fail "envsweep $e" ${O}_es.err
      python3 -c "
import json
d = json.load(open('${O}_es.json'))
print('[$e] value %.1f avg %.1f |' % (d['value'], d['avg_busbw']), ' '.join('%d:%.2f' % (s['bytes'], s['ms'] * 1e3) for s in d['sweep']), d['verified'],
      ' '.join('%s %.1f us' % (k, v.get('kernel_ms', 0) * 1e3) for k, v in d.get('schedules', {}).items()))
" | tee -a ${O}_envsweep.txt
    done ;;
  sweep)
    for L in $LIBS; do
      b=$(basename $L .so)
      MSCCL_AMD_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --pmc off --no-secondary \
        > ${O}_sweep2_$b.json 2>> ${O}_sweep.err || fail "sweep2 $L" ${O}_sweep.err
      MSCCL_AMD_LIB=$L timeout -k 10 300 python3 bench.py --vranks 8 --dtype fp16 --no-cpu --pmc off --no-secondary \
        > ${O}_sweep8_$b.json 2>> ${O}_sweep.err || fail "sweep8 $L" ${O}_sweep.err
      python3 -c "
import json
for k in ('2', '8'):
    d = json.load(open('${O}_sweep%s_$b.json' % k))
    print('$b', k, 'ranks: value %.1f avg %.1f |' % (d['value'], d['avg_busbw']), ' '.join('%d:%.2f' % (s['bytes'], s['ms'] * 1e3) for s in d['sweep']))
" | tee -a ${O}_sweep.txt
    done ;;
  *) fail "unknown step $step" ;;
  esac
done
echo "session done"
