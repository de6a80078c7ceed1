# Round-2 closing profiles: rocprofv3 kernel trace + PMC passes of every bench config line
set -o pipefail
for spec in "c2:c2" "c3:c3" "c4:c4" "c3w:c3 --word" "c4w:c4 --word" "c2off:c2 --offsets" "c3off:c3 --offsets"; do
  tag=${spec%%:*}; args=${spec#*:}
  bash tools/profile.sh r02f_$tag $args --pcie-sample-mib 0 > gpurun_out/profile_$tag.log 2>&1 || { tail -5 gpurun_out/profile_$tag.log; exit 1; }
  echo "$tag done"
done
