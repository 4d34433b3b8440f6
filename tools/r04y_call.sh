#!/bin/bash
# round-4 evidence after the train-step work and the small-root rule: GPU test suite, smoke, the
# interleaved A/B (head / round-3 kernels / full root scans), the default bench line
cd "$(dirname "$0")/.." || exit 2
exec bash tools/gpu_steps.sh \
  'gputests:600:python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread' \
  'smoke:200:python -u -c "import __graft_entry__ as g; g.smoke()"' \
  "ab:400:bash tools/ab_bench.sh 2 'noroot=--root-scan 0'" \
  "bench:600:python -u bench.py > gpurun_out/bench_r04y.json"
