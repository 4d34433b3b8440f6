#!/bin/bash
# Stages a copy of the production kernel sources with tools/diag_hooks.patch applied into
# /tmp/yk_hooks/csrc (the diagnostic stamps / ablation switches / yk_diag_* readers).  The
# diagnostic scripts compile from there; the production sources carry none of the hooks.
cd "$(dirname "$0")/.." || exit 2
set -e
rm -rf /tmp/yk_hooks && mkdir -p /tmp/yk_hooks
cp -r nypc-yacht-auction_amd/csrc /tmp/yk_hooks/csrc
patch -s -d /tmp/yk_hooks -p2 < tools/diag_hooks.patch
