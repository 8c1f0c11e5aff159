/**
 * MergeEncoder — TokenizerManager.encode (src/bpe/tokenizer/tokenizer-manager.js:13-61)
 * on the MI355X: the learned merges applied in rank order to the whole text.
 * encode(text) → { tokens, text, vocab, vocabStrings } as the reference's
 * (model = { vocab, vocabStrings, merges }).  Node 12 syntax.
 */
import { native } from './native.js';

export class MergeEncoder {
    constructor(engine, model) {
        this._engine = engine;
        this._model = model;
        const merges = model.merges || [];
        const flat = new Uint32Array(merges.length * 3);
        merges.forEach(function (m, i) { flat[3 * i] = m[0]; flat[3 * i + 1] = m[1]; flat[3 * i + 2] = m[2]; });
        this._h = native().bpeUpload(engine.device, flat);
    }

    encodeBytes(bytes) {
        return native().bpeEncode(this._engine.device, this._h, bytes);
    }

    async encode(text) {
        const bytes = new Uint8Array(Buffer.from(text, 'utf8'));
        const tokens = Array.from(this.encodeBytes(bytes));
        return { tokens: tokens, text: text, vocab: this._model.vocab, vocabStrings: this._model.vocabStrings };
    }
}
