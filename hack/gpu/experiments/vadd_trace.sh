# phase trace of 6 back-to-back hsa-vector-add runs (stderr), then 6 runs with an idle gap
for i in 1 2 3 4 5 6; do AMDKUBE_VADD_TRACE=1 timeout -k 5 30 ./amdkube/_native/bin/hsa-vector-add --json > /dev/null || exit 1; echo ---; done
for i in 1 2 3; do sleep 1; AMDKUBE_VADD_TRACE=1 timeout -k 5 30 ./amdkube/_native/bin/hsa-vector-add --json > /dev/null || exit 1; echo "--- (after 1 s idle)"; done
