#!/bin/bash
# The GPU evidence recipes (GPU box), one parameterised script in place of per-session run files.
# usage: tools/evidence.sh TAG RECIPE [RECIPE ...]   -> gpurun_out/<step>.log (+ files named below)
# Each recipe is one or more tools/gpu_steps.sh steps (own time limit; a timeout, abort or fault
# stops the call).  Variant libraries are prebuilt here into tools/_variants/NAME/ (tools/variant_lib.sh).
#   tests       pytest -m gpu (every GPU test), then __graft_entry__.smoke()
#   bench       python bench.py (the default line, every leg)      -> gpurun_out/bench_TAG.json
#   prof        tools/profile_bench.sh TAG: rocprofv3 kernel trace + FETCH/WRITE/MFMA passes
#   ab[:R[:V..]] tools/ab_bench.sh R (default 3) head vs base [vs variants V = NAME=FLAGS]
#   train       the AMP and the f32 train step times (tools/train_time.py, 512 examples)
#   trainab[:R[:amp|f32[:V,..]]] tools/train_ab.sh: head vs base [vs prebuilt variants V] train step
#   trainprof   rocprofv3 kernel trace of 30 AMP train steps (tools/prof_train.py) -> gpurun_out/trp_TAG/
#   divergence  the opt-in 256-game divergence statistic (tests/test_gpu_divergence.py)
#   fwdts       k_forward's phase stamps inside the engine (YK_TIMING build, tools/diag_fwd_prologue.py)
#   select      per-phase stamps of the descent / expansion (YK_SEL_TIMING build, tools/diag_select.py)
#   xspan       per-game launch spans of k_expand_backup (YK_XSPAN build, tools/diag_xspan.py)
#   amp         per-wave stamps of the AMP train step (YK_AMP_TIMING build, tools/diag_amp.py)
#   xlane       tools/_xlane_check: the DPP / permlane exchanges against __shfl_xor
#   dist2       2 gloo ranks sharing the GPU (tools/dist_rehearsal.sh) -> gpurun_out/dist2_TAG.json
#   spawn2      the same through bench.py's own launcher (--gpus 2, no torchrun) -> gpurun_out/spawn2_TAG.json
#   cores       bench.host_cores(): affinity mask, cgroup quota, OMP_NUM_THREADS of the box
# Example: tools/evidence.sh r05a tests bench prof ab:3:contract=-DXP_CONTRACT
cd "$(dirname "$0")/.." || exit 2
tag=$1
shift
[ -n "$tag" ] || { echo "usage: tools/evidence.sh TAG RECIPE..." >&2; exit 2; }
steps=()
for r in "$@"; do
  case "$r" in
    tests) steps+=("gputests:600:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf"
                   'smoke:200:python -u -c "import __graft_entry__ as g; g.smoke()"') ;;
    bench) steps+=("bench:600:python -u bench.py > gpurun_out/bench_$tag.json") ;;
    prof) steps+=("prof:900:bash tools/profile_bench.sh $tag") ;;
    ab*) IFS=: read -r _ rounds rest <<< "$r"
         steps+=("ab:900:bash tools/ab_bench.sh ${rounds:-3} ${rest//,/ }") ;;
    train) steps+=("t_amp:120:YK_AMP=1 python -u tools/train_time.py 512" "t_f32:120:python -u tools/train_time.py 512") ;;
    trainab*) IFS=: read -r _ rounds mode vars <<< "$r"
              steps+=("trainab:600:bash tools/train_ab.sh ${rounds:-3} ${mode:-amp} ${vars//,/ }") ;;
    trainprof) steps+=("trainprof:200:YK_AMP=1 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_$tag -o tr --output-format csv -- python3 tools/prof_train.py") ;;
    divergence) steps+=("divergence:400:YK_DIVERGENCE_STRIDE=16 YK_DIVERGENCE_TAG=$tag python -u -m pytest tests/test_gpu_divergence.py -x -q -s --timeout 380 --timeout-method thread") ;;
    fwdts) steps+=("fwdts:200:YK_LIB_PATH=tools/_variants/fwdts/libyacht_hip.so timeout -k 5 180 python -u tools/diag_fwd_prologue.py") ;;
    select) steps+=("select:200:YK_LIB_PATH=tools/_variants/sel/libyacht_hip.so timeout -k 5 180 python -u tools/diag_select.py") ;;
    xspan) steps+=("xspan:200:YK_LIB_PATH=tools/_variants/xspan/libyacht_hip.so timeout -k 5 180 python -u tools/diag_xspan.py") ;;
    amp) steps+=("amp_ts:120:YK_LIB_PATH=tools/_variants/amp/libyacht_hip.so python -u tools/diag_amp.py") ;;
    xlane) steps+=("xlane:60:tools/_xlane_check") ;;
    dist2) steps+=("dist2:600:bash tools/dist_rehearsal.sh > gpurun_out/dist2_$tag.json") ;;
    spawn2) steps+=("spawn2:600:python3 -u bench.py --gpus 2 --dist-backend gloo --envs 1024 --sims 25 --steps 1 --warmup 1 --coach-games 1024 --no-steady > gpurun_out/spawn2_$tag.json") ;;
    cores) steps+=('cores:60:python3 -c "import bench, json; print(json.dumps(bench.host_cores()))"') ;;
    *) echo "unknown recipe $r" >&2; exit 2 ;;
  esac
done
exec bash tools/gpu_steps.sh "${steps[@]}"
