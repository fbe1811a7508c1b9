cd $GRAFT_REPO_ROOT
for lib in libgsa libgsa_p2k8 libgsa_p2k4; do for tb in 64 128 256 512 1024 4096; do
GSA_LIB=$PWD/gpuseqalign_amd/$lib.so timeout -k 10 100 python tools/sparse_ab.py --variants pair2:4 --reps 5 --shapes 1024x100000 --tileBx $tb 2>/dev/null | sed "s/^/$lib /" | grep variant || exit 1
done; done
