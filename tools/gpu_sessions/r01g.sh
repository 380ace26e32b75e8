set -u
cd $GRAFT_REPO_ROOT
tools/gpu_check.sh r01g --steps 100 --warmup 10 --cpu-seconds 10 || exit $?
tools/gpu_pmc.sh r01g 2 "EncCT<2, 1>" 1610612736 || exit $?
tools/gpu_pmc.sh r01g 5 "EncCT<32, 32>" 2147483648 || exit $?
