#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-c5fit}"; mkdir -p "$OUT"; cd "$R" || exit 1
timeout -k 10 900 python -u tools/gpu/r5_c5fitdiag.py > "$OUT/diag.json" 2> "$OUT/diag.err" || { tail -5 "$OUT/diag.err"; exit 1; }
echo done
