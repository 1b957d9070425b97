# ring vs tree fallback latency (co-resident ranks)
set -o pipefail
for n in 2 8; do for b in 128 4096 65536 1048576 8388608; do for s in fbring fbtree; do
  timeout -k 5 60 python3 tools/lat_one.py --schedule $s --bytes $b --ranks $n --dtype 6 --iters 200 || exit 1
done; done; done
