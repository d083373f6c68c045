#!/bin/bash
# GPU box: tools/ps_time.py with the default library and each variant given (shredword_amd/<lib>)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
PAT=${PAT:-cl100k}
timeout -k 10 120 python3 "$R/tools/ps_time.py" $PAT || exit $?
for lib in "$@"; do
  SHREDWORD_HIP_LIB=$R/shredword_amd/$lib timeout -k 10 120 python3 "$R/tools/ps_time.py" $PAT || exit $?
done
