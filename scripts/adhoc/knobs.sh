cd $GRAFT_REPO_ROOT
ROUNDS=3 B32=1 OUT=r05_knobs VARIANTS="base=RDN_NOP=1;fall=RDN_BIG_FALL=1;wg160=RDN_WGLDS_BLOCKS=160" bash scripts/ab_env.sh > /dev/null 2>&1 || exit $?
