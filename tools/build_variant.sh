# Build libgpubpe.so from train.hip at git revision $1 (or "work" = the working
# tree) into gpu-bpe_amd/lib/$2/, with extra compiler flags $3 (e.g. -DGBPE_KTRACE);
# the other objects come from the working tree's build/.  For A/B runs via GBPE_LIB.
set -e
cd "$(dirname "$0")/../gpu-bpe_amd"
mkdir -p build/$2 lib/$2
if [ "$1" = work ]; then cp csrc/train.hip build/$2/train.hip; else git show "$1":gpu-bpe_amd/csrc/train.hip > build/$2/train.hip; fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $3 -Icsrc -I../include -c build/$2/train.hip -o build/$2/train.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/api.o build/$2/train.o build/encode.o build/pretok.o \
  build/host_io.o build/merge_encode.o -o lib/$2/libgpubpe.so
echo "lib/$2/libgpubpe.so"
