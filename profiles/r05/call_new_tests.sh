#!/bin/bash
# Round 5: the new GPU tests (shared context on two streams, INTEGRATION.md binding).
out=gpurun_out/${1:-r05a}
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py::test_context_shared_by_two_streams tests/test_integration_binding.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
exit $rc
