set -e
LIBS="fw2 fw8" bash tools/r06_ab.sh
