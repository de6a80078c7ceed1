#!/bin/bash
# ugrep_gpu with AddressSanitizer on the host (ugrep's sources and the drop-in
# adapter, integration/reflex_gpu_matcher.h; the reference libreflex and the
# engine's libraries uninstrumented -- their malloc/free/memcpy still go
# through the sanitizer's allocator and interceptors).  Build container only;
# output oracle/_ref/asan/ugrep_gpu_asan (git-ignored, travels to the GPU box).
set -e -o pipefail
cd "$(dirname "$0")/../.."
REF=/root/reference
R=oracle/_ref
O=$R/asan
mkdir -p $O
make -C oracle $PWD/$R/libreflex.a /tmp/ugrep_amd_dropin/ugrep.cpp > /dev/null
F="-O1 -g -fno-omit-frame-pointer -fsanitize=address -std=gnu++11 -msse2 -DHAVE_AVX512BW -DWITH_NO_INDENT \
   -DPLATFORM=\"x86_64-pc-linux-gnu\" -DGREP_PATH=\"/usr/bin\" -DHAVE_MMAP -DHAVE_STRUCT_DIRENT_D_TYPE \
   -DHAVE_STRUCT_DIRENT_D_INO -DHAVE_STAT_ST_ATIM -DHAVE_STAT_ST_MTIM -DHAVE_STAT_ST_CTIM -I$REF/include -w -pthread"
objs=""
for s in cnf glob output query screen stats vkey; do
  g++ $F -c $REF/src/$s.cpp -o $O/$s.o &
  objs="$objs $O/$s.o"
done
gcc -O1 -g -fsanitize=address -w -c $REF/src/zopen.c -o $O/zopen.o &
g++ $F -I$REF/src -Iintegration -Iinclude -c /tmp/ugrep_amd_dropin/ugrep.cpp -o $O/ugrep_gpu.o &
wait
g++ -fsanitize=address -pthread -o $O/ugrep_gpu_asan $O/ugrep_gpu.o $objs $O/zopen.o $R/libreflex.a \
    -Lugrep_amd -lugpu_host -ldl -Wl,-rpath,'$ORIGIN/../../../ugrep_amd'
ls -la $O/ugrep_gpu_asan
