set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -c "
import pytest, sys
rc = [int(pytest.main(['-q', '-m', 'gpu', 'tests/test_gpu_cnn.py', '-k', 'cfg3_two_tower', '-p', 'no:cacheprovider'])) for _ in range(5)]
print('rcs', rc)
sys.exit(max(rc))
" > gpurun_out/rep_t.log 2>&1 || { tail -30 gpurun_out/rep_t.log; exit 1; }
grep -E "passed|failed|rcs" gpurun_out/rep_t.log
echo DONE
