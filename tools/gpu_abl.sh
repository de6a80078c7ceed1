bash tools/pmc_lds.sh abl1 c4 libugrep_amd_abl1.so && bash tools/pmc_lds.sh abl2 c4 libugrep_amd_abl2.so && bash tools/gpu_sweep.sh abl c4 libugrep_amd_abl1.so libugrep_amd_abl2.so
