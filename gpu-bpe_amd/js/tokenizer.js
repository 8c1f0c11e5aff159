/**
 * TrieTokenizer — drop-in for the reference src/bpe/tokenizer/tokenizer.js
 * over the HIP chunked trie walk.  Chunk size: options.chunkSize, else
 * max(512, min(2048, maxTokenLen * 8)) (tokenizer.js:67-68); tokens never
 * cross a chunk; unmatched bytes map to their byte value.
 */
import { native } from './native.js';
import { compileVocabToTrie, parseHeader, parseTrieBuffers } from './trie.js';

const DEFAULT_CHUNK_SIZE = 512;
const UTF8_REPLACEMENT = [0xEF, 0xBF, 0xBD];

export class TrieTokenizer {
    constructor(engine, trieData, vocab, options) {
        this._engine = engine;
        const byteVocab = [];
        for (let i = 0; i < 256; i++) byteVocab.push([i]);
        this._vocab = vocab || byteVocab;
        const header = parseHeader(trieData);
        const bufs = parseTrieBuffers(trieData, header);
        this.nodeCount = header.nodeCount;
        this.edgeCount = header.edgeCount;
        this.maxTokenLen = header.maxTokenLen;
        const adaptive = Math.max(DEFAULT_CHUNK_SIZE, Math.min(2048, header.maxTokenLen * 8));
        this._chunkSize = options && options.chunkSize !== undefined && options.chunkSize !== null
            ? options.chunkSize : adaptive;
        this._trie = native().trieUpload(engine.device, bufs.nodes, bufs.edges);
        console.log('[ok] TrieTokenizer: ' + this.nodeCount + ' nodes, ' + this.edgeCount + ' edges, chunk=' +
            this._chunkSize);
    }

    static fromVocab(engine, vocab, options) {
        return new TrieTokenizer(engine, compileVocabToTrie(vocab), vocab, options || {});
    }

    get chunkSize() { return this._chunkSize; }

    async encodeBytes(bytes) {
        if (bytes.length === 0) return new Uint32Array(0);
        return native().encode(this._engine.device, this._trie, bytes, this._chunkSize);
    }

    decode(tokens) {
        let total = 0;
        const parts = [];
        for (const t of tokens) {
            const idx = Number(t);
            const b = idx < this._vocab.length ? this._vocab[idx] : UTF8_REPLACEMENT;
            parts.push(b);
            total += b.length;
        }
        const out = new Uint8Array(total);
        let off = 0;
        for (const p of parts) { out.set(p, off); off += p.length; }
        return out;
    }

    destroy() {
        if (this._trie) native().trieFree(this._trie);
        this._trie = null;
    }
}
