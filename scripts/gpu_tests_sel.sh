# Selected GPU test files (args), each file its own pytest run under a time limit; stops at the first failure.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "cpu: affinity $(python -c 'import os; print(len(os.sched_getaffinity(0)))') cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null) nproc $(nproc)"
for f in "$@"; do
  b=$(basename $f .py)
  timeout -k 10 900 python -u -m pytest $f -x -v -s --timeout 300 --timeout-method thread -rf > gpurun_out/$b.log 2>&1; rc=$?
  echo "$f rc=$rc"; tail -3 gpurun_out/$b.log
  [ $rc -eq 0 ] || exit $rc
done
