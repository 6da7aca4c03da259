cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for v in "$@"; do echo "== $v"; MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" MVS_BENCH_C4=1 timeout -k 10 200 python3 -u tools/kernel_bench.py 3 2>&1 | grep cfg || exit 1; done
