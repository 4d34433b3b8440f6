#!/bin/bash
# rocprofv3 evidence for bench.py (GPU box): kernel-trace stats of the bench command, then the
# HBM counters of k_forward and k_expand_backup in separate --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share a
# pass on gfx950), then k_forward's MFMA busy cycles.  usage: tools/profile_bench.sh TAG   -> gpurun_out/prof_TAG/
cd "$(dirname "$0")/.." || exit 2
set -e
export TMPDIR=/tmp
tag=${1:-r01}
out=gpurun_out/prof_$tag
mkdir -p $out
# the kernel sources measured (bench.py matches its roofline inputs to them)
python3 -c "import bench; print(bench.kernel_sources_sha16())" > $out/kernel_src_sha16.txt
args="--steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-coach --no-shape --no-f16 --no-train"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o bench --output-format csv -- python3 bench.py $args > $out/bench_trace.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --kernel-include-regex 'k_forward|k_expand_backup' --pmc $c -d $out/$c -o $c --output-format csv -- python3 bench.py $args --no-profile > $out/bench_$c.json
done
# MFMA utilisation of k_forward: busy cycles of the matrix pipes against the kernel's cycles
timeout -k 10 400 rocprofv3 --kernel-include-regex 'k_forward' --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  -d $out/MFMA -o MFMA --output-format csv -- python3 bench.py $args --no-profile > $out/bench_MFMA.json
python3 tools/summarize_prof.py $out > $out/summary.json
cat $out/summary.json
