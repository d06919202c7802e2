# import chunk lengths at light load: backward 16 ticks (DDR_CHUNK_BWD=16), forward 8 ticks (DDR_CHUNK_FWD=8)
cd $GRAFT_REPO_ROOT
LIBS="cur b16 f8" WLS="c3s8 light" TAG=r06_chunk bash tools/ktrace.sh
