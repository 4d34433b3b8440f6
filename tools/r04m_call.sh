#!/bin/bash
# round-4 final evidence (after the fused gradient norm): GPU test suite, smoke, the default bench
# line, and the bench's rocprofv3 kernel trace (tools/profile_bench.sh)
cd "$(dirname "$0")/.." || exit 2
exec bash tools/gpu_steps.sh \
  'gputests:600:python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread' \
  'smoke:200:python -u -c "import __graft_entry__ as g; g.smoke()"' \
  "bench:600:python -u bench.py > gpurun_out/bench_r04m.json" \
  "prof:900:bash tools/profile_bench.sh r04m"
