cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GSR_RENDER_QUAD=1 timeout -k 10 200 python tools/render_stats.py 32 || exit $?
GSR_RENDER_QUAD=3 timeout -k 10 200 python tools/render_stats.py 32 || exit $?
PIPE=avatar STEPS=100 timeout -k 10 900 bash tools/gpu_env_ab.sh GSR_RENDER_QUAD=0 GSR_QUAD_VARIANT=0 GSR_QUAD_VARIANT=1 GSR_QUAD_VARIANT=2 GSR_QUAD_VARIANT=3 || exit $?
