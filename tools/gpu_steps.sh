#!/bin/bash
# Sequential GPU steps for one gpurun call.  Each step runs under its own time limit;
# a test failure (exit 1) lets the next step run, anything else (fault, abort, segfault,
# time limit) ends the script there so nothing more touches the GPU in that call.
#   usage: tools/gpu_steps.sh <name> <seconds> <command...> [-- <name> <seconds> <command...>]...
# Each step's output goes to gpurun_out/<name>.log.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
final=0
while [ $# -gt 0 ]; do
  name=$1; secs=$2; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do cmd+=("$1"); shift; done
  [ "$1" = "--" ] && shift
  echo "[step] $name (limit ${secs}s): ${cmd[*]}"
  timeout -k 10 "$secs" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[step] $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[step] stopping after $name (rc=$rc)"
    exit $rc
  fi
  [ $rc -ne 0 ] && final=$rc
done
exit $final
