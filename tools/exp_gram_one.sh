cd $GRAFT_REPO_ROOT
VARIANTS=gram bash tools/exp_gram.sh
