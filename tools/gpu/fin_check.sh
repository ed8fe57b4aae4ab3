set -o pipefail
bash tools/gpu/diag_stage0.sh ablib/base.so ablib/fin.so ablib/diag1.so ablib/fin_diag1.so ablib/diag4.so && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fin.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fin.log; exit $rc
