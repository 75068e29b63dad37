#!/bin/bash
# Host-code sanitizer run (CPU only): the CPU test suite against ASan + UBSan
# builds of the oracle (oracle/_asan) and of libtsg's host code
# (spgemm_amd/lib/libtsg_asan.so; device code uninstrumented).  Python itself
# is not instrumented, so libasan is preloaded and leak reports are off.
# Host-only: run it in this container, not on the GPU box.
#   make -C oracle asan && make -C spgemm_amd/csrc asan && tools/asan_cpu.sh [pytest args]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
ASAN=$(gcc -print-file-name=libasan.so)
UBSAN=$(gcc -print-file-name=libubsan.so)
# appended: whatever is already preloaded stays first (hence verify_asan_link_order=0)
export LD_PRELOAD="${LD_PRELOAD:+$LD_PRELOAD }$ASAN $UBSAN"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:protect_shadow_gap=0:verify_asan_link_order=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export TSG_ORACLE_LIB=$ROOT/oracle/_asan/libtsg_oracle_asan.so
export TSG_LIB_PATH=$ROOT/spgemm_amd/lib/libtsg_asan.so
cd "$ROOT"
exec python -m pytest tests/test_oracle.py tests/test_lib_cpu.py -x -q -p no:cacheprovider "$@"
