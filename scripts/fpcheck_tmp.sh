set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/fpcheck2; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 200 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1; echo "$name done"; }
C="--config multivariate --steps 5 --warmup 2 --anomaly-frac 0"
run thr5_ewma8 $C --lstm-threshold 5 --lstm-cal-ewma 0.125
run thr4_pre800 $C --lstm-pretrain 800
run thr5_pre800 $C --lstm-threshold 5 --lstm-pretrain 800
run thr6 $C --lstm-threshold 6
run thr5_bf16 --config multivariate --steps 5 --warmup 2 --anomaly-frac 0 --lstm-threshold 5 --mv-bf16
timeout -k 10 400 python -u bench.py --config node > gpurun_out/node8.json 2> gpurun_out/node8.err || exit 1
