#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o kt -- python3 tools/prof_driver.py > gpurun_out/prof/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/prof/pA -o pA -- python3 tools/prof_driver.py --iters 2 > gpurun_out/prof/pA.log 2>&1
rc=$?; echo "pA rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv -d gpurun_out/prof/pB -o pB -- python3 tools/prof_driver.py --iters 2 > gpurun_out/prof/pB.log 2>&1
rc=$?; echo "pB rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pC -o pC -- python3 tools/prof_driver.py --iters 2 > gpurun_out/prof/pC.log 2>&1
rc=$?; echo "pC rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pD -o pD -- python3 tools/prof_driver.py --iters 2 > gpurun_out/prof/pD.log 2>&1
rc=$?; echo "pD rc=$rc"
ls -R gpurun_out/prof | head -50
exit 0
