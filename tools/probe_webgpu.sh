# C1 (BASELINE configs[0]): is there any WebGPU implementation on this box to run the
# reference on a software adapter (engine.js:143-177 requestGPUDevice)?  Records what exists.
echo "node: $(command -v node) $(node --version 2>/dev/null)"
echo "deno: $(command -v deno)  bun: $(command -v bun)"
for d in /usr/share/vulkan/icd.d /etc/vulkan/icd.d /usr/local/share/vulkan/icd.d; do echo "vulkan icd dir $d: $(ls $d 2>/dev/null | tr '\n' ' ')"; done
echo "libvulkan: $(ldconfig -p 2>/dev/null | grep -c libvulkan) entries"
echo "dawn/wgpu libs: $(ldconfig -p 2>/dev/null | grep -Eic 'dawn|wgpu_native|webgpu') entries"
echo "swiftshader/lavapipe: $(ls /usr/lib/x86_64-linux-gnu 2>/dev/null | grep -Eic 'swiftshader|lvp|vk_swiftshader') entries"
echo "chromium/chrome: $(command -v chromium chromium-browser google-chrome 2>/dev/null | tr '\n' ' ')"
node -e "console.log('node navigator.gpu:', typeof navigator !== 'undefined' && !!navigator.gpu)" 2>&1 | head -2
python3 -c "import importlib.util as u; print('python wgpu:', u.find_spec('wgpu') is not None)"
