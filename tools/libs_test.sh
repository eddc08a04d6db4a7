# One pytest selection per library build (SLAMGPU_LIB), each under its own time limit:
#   tools/libs_test.sh OUT "PYTEST_ARGS" lib1.so [lib2.so ...]
set -o pipefail
OUT=$1; ARGS=$2; shift 2
mkdir -p $OUT
for lib in "$@"; do
  n=$(basename $lib .so)
  SLAMGPU_LIB=$(readlink -f $lib) timeout -k 10 300 python3 -u -m pytest $ARGS -m gpu -q \
    --timeout 120 --timeout-method thread > $OUT/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(tail -1 $OUT/$n.log)"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
