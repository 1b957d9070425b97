# ring / chain tree / flat tree fallback latency (co-resident ranks), fp16: device time per launch
# from a hipGraph replay of back-to-back launches (tools/lat_one.py --graph), then per call through
# Python
set -o pipefail
for n in ${RANKS:-2 8}; do for b in ${BYTES:-128 4096 65536}; do for s in fbring fbchain fbtree; do
  timeout -k 5 60 python3 tools/lat_one.py --schedule $s --bytes $b --ranks $n --dtype 6 --iters 200 --graph || exit 1
done; done; done
