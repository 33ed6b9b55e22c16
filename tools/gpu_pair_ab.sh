set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "pair" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02f_pytest.log 2>&1; echo PYTEST=$?; tail -3 gpurun_out/r02f_pytest.log
for L in 1 2; do
timeout -k 10 300 python bench.py --config C3 --steps 2 --warmup 1 --cpu-baseline 0 --lanes-per-pixel $L > gpurun_out/r02f_c3_l$L.json 2>gpurun_out/r02f_c3_l$L.err || { echo "bench L=$L failed"; tail -3 gpurun_out/r02f_c3_l$L.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' gpurun_out/r02f_c3_l$L.json L$L
done
