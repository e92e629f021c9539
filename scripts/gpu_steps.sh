# Run GPU steps in order; stop at the first crash-like exit (fault, abort,
# timeout), keep going after ordinary test failures.
#   bash scripts/gpu_steps.sh "name:seconds:command" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 $secs bash -c "$cmd" > gpurun_out/$name.log 2>&1
  rc=$?
  echo "step $name rc=$rc"; tail -3 gpurun_out/$name.log
  case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
done
