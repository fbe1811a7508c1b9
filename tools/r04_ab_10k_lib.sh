# same-box A/B of the 10k full fill (fused, unpadded) between the default build and a diagnostic build
# (GSA_LIB=$1), alternated
set -e
for r in 1 2 3; do
  for L in "" "$1"; do
    echo "lib ${L:-default}"; GSA_LIB=$L timeout -k 10 100 python -u tools/full_ab.py --batch 0 --rounds 1 2>/dev/null | grep '"pitched": false'
  done
done
