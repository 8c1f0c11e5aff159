# Kernel resource usage (VGPRs, scratch, occupancy) of the training unit's k_body /
# k_refresh instances, from the compiler's remarks: tools/ru.sh [tree root]
R=${1:-$(dirname "$0")/..}
cd "$R/gpu-bpe_amd" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc -I../include \
  -c csrc/train.hip -o /tmp/ru_train.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 "$(cd "$OLDPWD" && cd "$(dirname "$0")" && pwd)/ru_parse.py"
