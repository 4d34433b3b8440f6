#!/bin/bash
# round-4 evidence, part 1: the GPU test suite, smoke, and the rocprofv3 kernel trace + PMC passes
cd "$(dirname "$0")/.." || exit 2
exec bash tools/gpu_steps.sh \
  'gputests:600:python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread' \
  'smoke:200:python -u -c "import __graft_entry__ as g; g.smoke()"' \
  "prof:900:bash tools/profile_bench.sh r04z"
