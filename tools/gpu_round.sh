#!/bin/bash
# GPU evidence for one bench configuration: rocprofv3 kernel stats + PMC passes of
# the workload (tools/profile.sh), the summary and the kernel-stats CSV copied
# into profiles/, then the bench itself (its roofline reads that summary).
# Usage: bash tools/gpu_round.sh TAG NAME [bench args]
#   e.g. bash tools/gpu_round.sh r02 c2            (the default bench line)
#        bash tools/gpu_round.sh r02 c3 --config C3
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}; NAME=${2:-c2}; shift 2
ARGS="$@"
mkdir -p gpurun_out
bash tools/profile.sh ${TAG}_$NAME --steps 1 --warmup 0 --cpu-baseline 0 --fast-extra 0 $ARGS > gpurun_out/profile_${TAG}_$NAME.log 2>&1 || { echo PROFILE FAILED; tail -5 gpurun_out/profile_${TAG}_$NAME.log; exit 1; }
mkdir -p gpurun_out/stage_profiles && cp gpurun_out/prof_${TAG}_$NAME/summary.json gpurun_out/stage_profiles/${TAG}_pmc_summary_$NAME.json
f=$(ls gpurun_out/prof_${TAG}_$NAME/ktrace/*/*kernel_stats.csv gpurun_out/prof_${TAG}_$NAME/ktrace/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/stage_profiles/${TAG}_kernel_stats_$NAME.csv
python3 -c 'import json,sys; s=json.load(open(sys.argv[1])); print({k: s.get(k) for k in ("avg_duration_ms","serialized_avg_duration_ms","effective_clock_ghz","valu_issue_frac_serialized","valu_lane_utilization","sq_wait_any_frac","l2_hit_rate","hbm_bytes_per_launch","lds_bank_conflict_cycles_per_lds_inst","ta_accesses_per_cu_cycle","launches_per_step")})' gpurun_out/stage_profiles/${TAG}_pmc_summary_$NAME.json
