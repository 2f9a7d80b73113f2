#!/bin/bash
# Round-5 blur A/B: the main library against milwrm_amd/lib_<V>.so for V in
# $VARIANTS: blur-only timing (tools/blur_bench.py, a strided sample of the
# output saved per library and compared), the config-2 bench and (C5=1) the
# config-5 slice, alternating; then the blur parity tests on the main library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-blurab}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
summ='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["ms_per_step"],2), {k:round(v["total_ms_per_step"],2) for k,v in d["kernels"].items()})'
for r in 1 2; do
  for v in main $VARIANTS; do
    L=""; [ $v = main ] || L="$GRAFT_REPO_ROOT/milwrm_amd/lib_$v.so"
    timeout -k 10 120 env ${L:+MW_LIB=$L} BLUR_SAVE=$OUT/blur_$v.npy python tools/blur_bench.py 10000 30 "" > $OUT/bb_$v.txt 2>&1 || { tail -3 $OUT/bb_$v.txt; exit 1; }
    echo "blur $v: $(cat $OUT/bb_$v.txt | tail -1)"
    timeout -k 10 120 env ${L:+MW_LIB=$L} BLUR_SAVE=$OUT/blur50_$v.npy python tools/blur_bench.py 6000 50 "" > $OUT/bb50_$v.txt 2>&1 || { tail -3 $OUT/bb50_$v.txt; exit 1; }
    echo "blur50 $v: $(cat $OUT/bb50_$v.txt | tail -1)"
  done
done
python -c "
import numpy as np, sys
for v in sys.argv[1:]:
    for c in ('', '50'):
        a=np.load('$OUT/blur%s_main.npy'%c); b=np.load('$OUT/blur%s_%s.npy'%(c,v))
        print('bitwise main vs', v, c or '30', a.view(np.uint32).tobytes()==b.view(np.uint32).tobytes())
" $VARIANTS
for r in $(seq 1 ${C2:-2}); do
  for v in main $VARIANTS; do
    L=""; [ $v = main ] || L="$GRAFT_REPO_ROOT/milwrm_amd/lib_$v.so"
    timeout -k 10 200 env ${L:+MW_LIB=$L} $BENV python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2_$v.json 2> $OUT/c2_$v.err || { tail -3 $OUT/c2_$v.err; exit 1; }
    python -c "$summ" $OUT/c2_$v.json "c2 $v"
  done
done
for r in $(seq 1 ${C5:-0}); do
  for v in main $VARIANTS; do
    L=""; [ $v = main ] || L="$GRAFT_REPO_ROOT/milwrm_amd/lib_$v.so"
    timeout -k 10 300 env ${L:+MW_LIB=$L} $BENV python bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail -3 $OUT/c5_$v.err; exit 1; }
    python -c "$summ" $OUT/c5_$v.json "c5 $v"
  done
done
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  rc=$?; tail -2 $OUT/pytest.log; grep -E "^FAILED|^ERROR" $OUT/pytest.log | head; [ $rc -eq 0 ] || exit $rc
fi
echo "[blurab] done"
