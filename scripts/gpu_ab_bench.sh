# Same-box flagship A/B: bash scripts/gpu_ab_bench.sh OUT "ENV_A" "ENV_B" [rounds] [bench args]
# alternates bench.py runs with env assignments A and B (e.g. "DA_BLAS_PREFILL=1" "DA_BLAS_PREFILL=0").
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/$1; A=$2; B=$3; N=${4:-2}; shift 4 || true
ARGS="$@"
mkdir -p $OUT
for i in $(seq 1 $N); do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 400 python bench.py --steps 4 --warmup 1 --latency-reps 3 --ingest-docs 0 $ARGS > $OUT/${arm}_$i.json 2> $OUT/${arm}_$i.err || { tail -5 $OUT/${arm}_$i.err; exit 1; }
    echo "$arm[$E] $(python -c "import json,sys; d=json.load(open('$OUT/${arm}_$i.json')); print(d['value'], d['ms_per_step'], d.get('p50_cache_miss_ms'))")"
  done
done
