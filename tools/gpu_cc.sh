#!/bin/bash
# coefficient rate parity + the TPL / motion rows touched this round
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_costcoeffs.py tests/test_gpu_rdo_rate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_cc.log 2>&1; rc=$?; echo "cc rc=$rc"; tail -3 gpurun_out/pytest_cc.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_tpl.sh || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_mcomp_fixtures.py tests/test_gpu_mcomp.py tests/test_gpu_subpel.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_mot.log 2>&1; rc=$?; echo "mot rc=$rc"; tail -3 gpurun_out/pytest_mot.log; exit $rc
