set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 240 python bench.py --vranks 8 --dtype fp16 --no-cpu --pmc off --steps 20 --warmup 5 > $O/r06c_c3_new.json 2> $O/r06c_c3_new.err &&
MSCCL_AMD_LOWER_LARGE=0 timeout -k 10 240 python bench.py --vranks 8 --dtype fp16 --no-cpu --pmc off --steps 20 --warmup 5 > $O/r06c_c3_old.json 2> $O/r06c_c3_old.err &&
timeout -k 10 240 python bench.py --no-cpu --pmc off --steps 20 --warmup 5 > $O/r06c_c2_new.json 2> $O/r06c_c2_new.err &&
MSCCL_AMD_LOWER_LARGE=0 timeout -k 10 240 python bench.py --no-cpu --pmc off --steps 20 --warmup 5 --sizes 33554432 > $O/r06c_c2_old.json 2> $O/r06c_c2_old.err
