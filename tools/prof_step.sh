#!/bin/bash
# rocprofv3 kernel-trace stats of one command: prof_step.sh <out-dir-name> <command...>
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
name=$1; shift
cd /tmp && exec rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$name" -o k -- "$@"
