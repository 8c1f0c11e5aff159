// Loads the N-API addon (gpubpe.node, built by `make -C gpu-bpe_amd addon`).
// There is no fallback: without the addon / a HIP device every entry point throws.
import { createRequire } from 'module';

const require = createRequire(import.meta.url);
let addon = null;
let loadError = null;
try {
    addon = require('./gpubpe.node');
} catch (e) {
    loadError = e;
}

export function native() {
    if (!addon) {
        throw new Error('gpubpe native addon not available (' + (loadError ? loadError.message : 'unknown') +
            '); build it with `make -C gpu-bpe_amd addon`');
    }
    return addon;
}
