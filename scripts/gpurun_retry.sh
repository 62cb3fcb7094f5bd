# Run one gpurun call, retrying ONLY when no box / slot was free (exit 3, nothing ran, nothing charged).
# usage: bash scripts/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1; rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box\|slots on this pod are busy\|backing off\|stopped responding while being prepared\|taken away by the GPU service\|has no free box" $out; then exit $rc; fi
  sleep 150
done
exit $rc
