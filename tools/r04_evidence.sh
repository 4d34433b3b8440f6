#!/bin/bash
# round-4 measurements on the GPU box (prebuilt variant libraries under tools/_variants/):
#   ab        interleaved A/B: head, the round-3 kernels (base), head without the incremental root
#             scan (--root-scan 0), head built with -mllvm -disable-machine-licm (nolicm)
#   diverge   the bench-size self-play test with accurate expf/logf in the softmax (ieeexp variant):
#             its divergence statistic against an independent f32 oracle run
#   sel       per-phase cycles of the descent / expansion (YK_SEL_TIMING variant)
#   xspan     k_expand_backup launch span vs per-game times (YK_XSPAN variant)
#   trunk     the k_forward timing harness with per-wave stamps of one residual block
#   prof      rocprofv3 kernel trace + HBM / MFMA counters of the bench (tools/profile_bench.sh)
cd "$(dirname "$0")/.." || exit 2
tag=${1:-r04a}
exec bash tools/gpu_steps.sh \
  "ab:300:bash tools/ab_bench.sh 2 'noroot=--root-scan 0' nolicm=x" \
  "diverge:200:YK_LIB_PATH=tools/_variants/ieeexp/libyacht_hip.so python -u -m pytest tests/test_gpu_selfplay.py -k bench_size -x -q -s --timeout 180 --timeout-method thread" \
  "sel:200:YK_LIB_PATH=tools/_variants/sel/libyacht_hip.so timeout -k 5 180 python -u tools/diag_select.py" \
  "xspan:200:YK_LIB_PATH=tools/_variants/xspan/libyacht_hip.so timeout -k 5 180 python -u tools/diag_xspan.py" \
  "trunk:60:timeout -k 5 50 ./tools/_abl_t 3480" \
  "prof:600:bash tools/profile_bench.sh $tag"
