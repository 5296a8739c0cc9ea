cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_pmc
PMC_OUT=gpurun_out/r05_pmc bash scripts/pmc.sh python bench.py --pmc-child --no-cpu-baseline --steps 2 --warmup 1 --batch 16
