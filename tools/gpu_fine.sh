set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fine1
SR_FINE=1 SERIATION_LIB=seriation-in-paleontological-data-using-mcmc_amd/build/var/fine/libseriation.so timeout -k 10 120 python tools/stamp_profile.py > gpurun_out/fine1/fine.log 2>&1
cat gpurun_out/fine1/fine.log
