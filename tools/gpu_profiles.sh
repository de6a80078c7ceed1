# Round profiles: rocprofv3 kernel trace + PMC passes of the C2/C3/C4 bench configs
set -o pipefail
for c in c2 c3 c4; do
  PMC3=1 bash tools/profile.sh r02_$c $c --pcie-sample-mib 0 > gpurun_out/profile_$c.log 2>&1 || exit 1
done
