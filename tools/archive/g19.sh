set -uo pipefail
for L in prof x1 x2; do echo "== $L"; TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_$L.so timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | tail -4 || exit 1; done
