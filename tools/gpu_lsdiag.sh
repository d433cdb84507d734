#!/bin/bash
# config-3 end-to-end deviation over many seeds: this build vs ablib/old.so (previous order)
export TMPDIR=/tmp
mkdir -p gpurun_out
SEEDS=${SEEDS:-48} timeout -k 10 400 python -u tools/diag_ls_e2e.py 1 > gpurun_out/lsdiag_new.log 2>&1
rc=$?
tail -1 gpurun_out/lsdiag_new.log
[ $rc -ne 0 ] && exit $rc
SEEDS=${SEEDS:-48} LGS_LIB=ablib/old.so timeout -k 10 400 python -u tools/diag_ls_e2e.py 1 > gpurun_out/lsdiag_old.log 2>&1
rc=$?
tail -1 gpurun_out/lsdiag_old.log
exit $rc
