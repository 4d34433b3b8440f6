#!/bin/bash
# GPU box: the round's evidence - the GPU test suite, the default bench line (all legs), and the
# rocprofv3 kernel trace + HBM counters of the bench configuration (tools/profile_bench.sh).
# usage: tools/final_evidence.sh TAG  -> gpurun_out/gputests.log, gpurun_out/bench_TAG.json, gpurun_out/prof_TAG/
cd "$(dirname "$0")/.." || exit 2
tag=${1:-r01}
exec bash tools/gpu_steps.sh \
  'gputests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
  "bench:400:python -u bench.py > gpurun_out/bench_$tag.json" \
  "prof:900:bash tools/profile_bench.sh $tag"
