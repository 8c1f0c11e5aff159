/**
 * BPEEngine — MI355X device bring-up over the gpubpe C-ABI.
 *
 * Drop-in for the reference src/bpe/engine.js: same exported constants
 * (engine.js:10-22), same class surface (init / device / pipelines /
 * limits, engine.js:181-245).  `device` is an opaque context handle and
 * `pipelines` a name-keyed object of the native kernels (bpe-worker.js
 * logs its key count).  Node 12 syntax (no ?. ?? or private methods).
 */
import { native } from './native.js';

export const WORKGROUP_SIZE = 256;
export const TABLE_SIZE = 2097152;
export const INVALID_TOKEN = 0xFFFFFFFF;
export const MAX_WG_DIM = 65535;

const MB = 1024 * 1024;
export const GPU_LIMITS = Object.freeze({
    MAX_STORAGE_BUFFER_SIZE: 512 * MB,
    MAX_BUFFER_SIZE: 512 * MB,
    MAX_COMPUTE_WORKGROUPS_PER_DIM: MAX_WG_DIM,
});

/** Kept for API compatibility (engine.js:37-48); HIP grids need no 2D split. */
export function dispatch2D(pass, totalWorkgroups) {
    if (totalWorkgroups <= 0) return;
    if (totalWorkgroups <= MAX_WG_DIM) { pass.dispatchWorkgroups(totalWorkgroups); return; }
    const x = Math.min(totalWorkgroups, MAX_WG_DIM);
    pass.dispatchWorkgroups(x, Math.ceil(totalWorkgroups / x));
}

export class BPEEngine {
    constructor(options) {
        this._deviceIndex = options && typeof options.device === 'number' ? options.device : 0;
        this._ctx = null;
        this._pipelines = {};
        this._limits = null;
        this._initialized = false;
    }

    get device() { this._assertInitialized(); return this._ctx; }
    get pipelines() { this._assertInitialized(); return this._pipelines; }
    get limits() { this._assertInitialized(); return this._limits; }

    async init() {
        if (this._initialized) return this;
        const n = native();
        this._ctx = n.createContext(this._deviceIndex);
        const lim = n.limits(this._ctx);
        this._limits = { maxBufferSize: lim.maxBufferSize };
        const names = n.kernelNames();
        const p = {};
        for (const k of names) p[k] = k;
        this._pipelines = p;
        this._initialized = true;
        console.log('[ok] BPE Engine initialized (' + names.length + ' kernels, MI355X/HIP)');
        return this;
    }

    destroy() {
        if (this._ctx) native().destroyContext(this._ctx);
        this._ctx = null;
        this._initialized = false;
    }

    _assertInitialized() {
        if (!this._initialized) {
            throw new Error('BPEEngine not initialized — call await engine.init() first');
        }
    }
}
