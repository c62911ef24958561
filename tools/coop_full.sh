# coop-kernel iteration with stamps: parity suite, bench lines at 8,192 / 4,096 roots, then the
# diagnostic build's phase stamps (LIBS, default libmzh_diag.so).  SKIP_TESTS=1: timing only
set -e
SKIP_TESTS=${SKIP_TESTS:-} bash tools/coop_iter.sh
LIBS=${LIBS:-muzero-hanoi_amd/libmzh_diag.so} bash tools/stamp_ab.sh
