# Round-2 second-session profiles: xc_kernel (C3), xc_kernel with W (C3 -w), \w+ under W (C4 -w)
set -o pipefail
bash tools/profile.sh r02_c3xc c3 --pcie-sample-mib 0 > gpurun_out/profile_c3xc.log 2>&1 || exit 1
bash tools/profile.sh r02_c3w c3 --word --pcie-sample-mib 0 > gpurun_out/profile_c3w.log 2>&1 || exit 1
bash tools/profile.sh r02_c4w c4 --word --pcie-sample-mib 0 > gpurun_out/profile_c4w.log 2>&1 || exit 1
