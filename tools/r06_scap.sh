# C5 piece split threshold (percent of the block capacity; 80 for a dominant basin): 60 / 70 / 90 against the build
cd $GRAFT_REPO_ROOT
LIBS="cur scap60 scap70 scap90" WLS="c5" TAG=r06_scap bash tools/ktrace.sh
