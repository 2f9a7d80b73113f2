#!/bin/bash
# Round-4 GPU pass 2: full-size M-step checks, configs 3/4 at full per-rank
# size, config-5 cohort / sweep / host-source bench lines, rocprof of config 2.
set -o pipefail
TAG=${1:-r4b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
C5="--size 40000 --channels 50 --slides-per-gpu 2 --source synth --steps 2 --warmup 1 --no-cpu-baseline"
true && \
timeout -k 10 1000 python -u -m pytest tests/test_gpu_config34.py -x -v -s --timeout 1000 $T -m gpu > $OUT/config34.log 2>&1 && \
timeout -k 10 300 python -u bench.py $C5 > $OUT/bench_c5x2_synth.json 2> $OUT/bench_c5x2_synth.err && \
MW_LLOYD_FIRST_W2=1 timeout -k 10 300 python -u bench.py $C5 > $OUT/bench_c5x2_synth_w2.json 2> $OUT/bench_c5x2_synth_w2.err && \
timeout -k 10 300 python -u bench.py --sweep --steps 3 --warmup 1 > $OUT/bench_sweep10k.json 2> $OUT/bench_sweep10k.err && \
timeout -k 10 300 python -u bench.py --sweep --size 20000 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_sweep20k.json 2> $OUT/bench_sweep20k.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c2 -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err && \
timeout -k 10 600 python -u bench.py --size 40000 --channels 50 --slides-per-gpu 1 --source host --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_host.json 2> $OUT/bench_c5_host.err
