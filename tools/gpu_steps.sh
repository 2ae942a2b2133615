#!/bin/bash
# Run GPU steps in order on the box; each step is "<seconds> <command...>"
# on its own line of the file given as $1.  A step that fails plainly
# (exit 1: a test failure) does not stop the run; a time limit (124 / 137),
# an abort (134), a segfault (139) or any other status does: nothing more
# touches the GPU after it.
#   bash tools/gpu_steps.sh <steps-file>
set -u
while IFS= read -r line || [ -n "$line" ]; do
    [ -z "$line" ] && continue
    case "$line" in \#*) continue ;; esac
    secs=${line%% *}
    cmd=${line#* }
    echo "[gpu_steps $(date +%H:%M:%S)] ($secs s) $cmd"
    timeout -k 10 "$secs" bash -c "$cmd"
    rc=$?
    echo "[gpu_steps $(date +%H:%M:%S)] rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "[gpu_steps] stopping: rc=$rc"
        exit $rc
    fi
done < "$1"
