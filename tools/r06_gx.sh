# q' gather variants at C5 (kernel traces): base, 1-D grid, XCD-aware workgroup mapping (chunks of 4, 2, 8 tiles)
cd $GRAFT_REPO_ROOT
LIBS="base cur" WLS="c5" TAG=r06_gx bash tools/ktrace.sh
