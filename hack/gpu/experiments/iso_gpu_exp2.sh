#!/bin/bash
B=amdkube/_native/bin
H=hack/gpu/experiments/hsa_status
R=$(ls /dev/dri/renderD* | head -1)
run() { echo "== $1"; shift; env -u ROCR_VISIBLE_DEVICES -u HIP_VISIBLE_DEVICES timeout -k 5 60 "$@" 2>&1 | tail -4; echo "rc=${PIPESTATUS[0]}"; }
run "baseline" $H
run "keep $R" $B/amdkube-nsexec --no-namespaces --landlock --keep $R -- $H
run "render denied (EACCES), kfd allowed" $B/amdkube-nsexec --no-namespaces --landlock -- $H
run "render + kfd denied" $B/amdkube-nsexec --no-namespaces --landlock --hide-kfd -- $H
ls -la /dev/dri/ /sys/class/kfd/kfd/topology/nodes/ 2>&1 | head -30
grep -l "drm_render_minor" /sys/class/kfd/kfd/topology/nodes/*/properties | head; grep -h drm_render_minor /sys/class/kfd/kfd/topology/nodes/*/properties
