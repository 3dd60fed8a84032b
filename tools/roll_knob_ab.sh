# A/B of the rolling conv's environment knobs on the cfg-2 EDSR / DUF steps
cd $GRAFT_REPO_ROOT
run() { echo "== $*"; env "$@" timeout -k 10 300 python bench.py --models edsr,duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (round(v['ms_per_step'],3), {a: round(b['ms_per_step'],3) for a,b in v['roofline']['by_direction'].items()}) for k,v in d['models'].items()})" || exit 1; }
run X=0
run VSRK_ROLL_PRIO=1
run VSRK_ROLL_WRES=0
run X=0
