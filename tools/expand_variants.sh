#!/bin/bash
# diagnostic: bench kernel times for expand-kernel build variants (GPU box)
cd "$(dirname "$0")/.." || exit 2
set -e
for v in "" "-DYK_EXPAND_WPE=3"; do
  make -s -C nypc-yacht-auction_amd clean > /dev/null
  make -s -C nypc-yacht-auction_amd EXTRA="$v" > /dev/null
  echo "[$v]"
  timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-train 2>/dev/null | \
    python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(round(d['value']/1e6,2), 'M exp/s', {k: v['avg_ms'] for k, v in d['kernel_ms'].items()})"
done
make -s -C nypc-yacht-auction_amd clean > /dev/null && make -s -C nypc-yacht-auction_amd > /dev/null
