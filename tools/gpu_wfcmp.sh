#!/bin/bash
# Wavefront variant against the megakernel at C2, C4, C5 (reduced spp: the wavefront
# takes seconds per frame): bench lines of both, PMC summaries of both (k_trace;
# k_wf_trace and k_wf_logic).  Usage: bash tools/gpu_wfcmp.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05wc}
mkdir -p gpurun_out
for cs in "C2 64" "C4 256" "C5 32"; do
  set -- $cs; C=$1; S=$2
  for v in mega wf; do
    W=""; [ $v = wf ] && W="--wavefront"
    A="--config $C --spp $S --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 --fast-extra 0 $W"
    o=gpurun_out/${TAG}_${C}_$v
    timeout -k 10 600 python bench.py $A > $o.json 2> $o.err || { echo "$C $v bench FAILED"; tail -5 $o.err; exit 1; }
    python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], sys.argv[3], d["ms_per_step"], "ms", d["value"], "Mrays/s", d["phases_ms_per_step"]["trace"], "trace ms")' $o.json $C $v
    bash tools/profile.sh ${TAG}_${C}_$v $A > /dev/null || { echo "$C $v profile FAILED"; exit 1; }
    if [ $v = wf ]; then
      python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_${C}_$v k_wf_trace > gpurun_out/prof_${TAG}_${C}_$v/summary_trace.json
      python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_${C}_$v k_wf_logic > gpurun_out/prof_${TAG}_${C}_$v/summary_logic.json
    fi
  done
done
