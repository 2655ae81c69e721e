set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=/tmp/bav_ht
rm -rf $D && mkdir -p $D && cp -r $R/slam-indoor-code_amd/slamhip $D/
cp $R/scripts/diag/lib_diag_ht.so $D/slamhip/libslamhip.so
sed "s#sys.path.insert(0, os.path.join(ROOT, \"slam-indoor-code_amd\"))#sys.path.insert(0, \"$D\")#" $R/scripts/ba_bench.py > $D/ba_bench.py
timeout -k 5 90 python3 $D/ba_bench.py 8 10000 > $R/gpurun_out/ht_w8.log 2>&1 && timeout -k 5 90 python3 $D/ba_bench.py 16 40000 4k > $R/gpurun_out/ht_w16.log 2>&1
