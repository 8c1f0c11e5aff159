/**
 * GpuPreTokenizer — the reference PreTokenizer (src/wasm/pre_tokenizer.mjs:402-509)
 * with its GPT-4 word-boundary rules computed on the MI355X.
 *
 * preTokenizeBytes(bytes) / preTokenize(text) return { bytes, wordStarts } like
 * the reference; BPETrainer.train(input, { preTokenizer }) accepts it the same
 * way (trainer.js:62-99).  Input must already be NFC (the reference
 * NFC-normalises first, which leaves NFC text unchanged).  Node 12 syntax.
 */
import { native } from './native.js';

export class GpuPreTokenizer {
    constructor(engine) {
        if (!engine) throw new Error('GpuPreTokenizer requires an initialized BPEEngine');
        this._engine = engine;
    }

    preTokenizeBytes(rawBytes) {
        if (!rawBytes || rawBytes.length === 0) return { bytes: new Uint8Array(0), wordStarts: new Uint8Array(0) };
        const bytes = rawBytes instanceof Uint8Array ? rawBytes : new Uint8Array(rawBytes);
        const wordStarts = native().pretokenizeGpt4(this._engine.device, bytes);
        return { bytes, wordStarts };
    }

    preTokenize(text) {
        if (!text || text.length === 0) return { bytes: new Uint8Array(0), wordStarts: new Uint8Array(0) };
        return this.preTokenizeBytes(new Uint8Array(Buffer.from(text, 'utf8')));
    }
}
