set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/pytest_gpu4.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu4.log
FLAGS=0 bash tools/variants.sh > gpurun_out/variants2.log 2>&1; cat gpurun_out/variants2.log
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo LIST=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ktrace -o run --output-format csv -- python bench.py --spp 64 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_ktrace.log 2>&1; echo KTRACE=$?
find gpurun_out/prof_ktrace -name "*stats*" | head
