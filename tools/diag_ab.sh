cd $GRAFT_REPO_ROOT
for L in ${LIBS:-libhipgp libhipgp_ct256}; do echo "== $L"; HGP_LIB=$PWD/hipgp_amd/$L.so timeout -k 10 300 python tools/diag_contig.py ${SHAPES:-1025x8 2048x8 4096x8 2100x8 8x2048} || exit 1; done
