#!/bin/bash
# one rocprofv3 PMC pass (kernel filter + counters) of one command:
#   pmc_step.sh <out-dir-name> <kernel-regex> "<counters>" <command...>
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
name=$1; rx=$2; ctr=$3; shift 3
cd /tmp && exec rocprofv3 --kernel-include-regex "$rx" --pmc $ctr --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$name" -o p -- "$@"
