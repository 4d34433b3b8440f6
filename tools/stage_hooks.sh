#!/bin/bash
# Stages a copy of the production kernel sources with the diagnostic hooks inserted
# (tools/diag_sources.py: stamps and yk_diag_* readers under their -DYK_* switches) into
# /tmp/yk_hooks/csrc.  The diagnostic scripts compile from there; the production sources carry
# none of the hooks.
cd "$(dirname "$0")/.." || exit 2
set -e
python3 tools/diag_sources.py /tmp/yk_hooks > /dev/null
