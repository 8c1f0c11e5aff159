# Build libgpubpe.so with extra compiler flags $2 (e.g. -DGBPE_KTRACE) into
# gpu-bpe_amd/lib/$1/, from the working tree (the training units recompiled,
# the other objects from build/).  For A/B runs via GBPE_LIB.
set -e
cd "$(dirname "$0")/../gpu-bpe_amd"
mkdir -p build/$1 lib/$1
for u in train train_lexshard; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $2 -Icsrc -I../include -c csrc/$u.hip -o build/$1/$u.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/api.o build/$1/train.o \
  build/$1/train_lexshard.o build/encode.o build/pretok.o build/host_io.o build/merge_encode.o -o lib/$1/libgpubpe.so
echo "lib/$1/libgpubpe.so"
