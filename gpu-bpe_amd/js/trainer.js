/**
 * BPETrainer — drop-in for the reference src/bpe/trainer.js over the HIP
 * merge loop.  train(input, {targetVocabSize = 4096, preTokenizer = null,
 * onProgress = null, wordStarts = null}) resolves to {vocab, vocabStrings,
 * vocabSize, merges: [a, b, id][], trainingTime} (trainer.js:328-334).  One
 * native step per batch of 128 merges (training-pipeline.js:13); onProgress
 * fires once per batch with the reference's fields (trainer.js:306-315).
 * The Vocab persists across train() calls (trainer.js:136, 191).
 */
import { native } from './native.js';
import { Vocab } from './vocab.js';

export const BATCH_SIZE = 128;

function formatDuration(seconds) {
    if (seconds < 60) return seconds.toFixed(1) + 's';
    const m = Math.floor(seconds / 60);
    const s = Math.round(seconds % 60);
    return s > 0 ? m + 'm ' + s + 's' : m + 'm';
}

function nowMs() {
    const t = process.hrtime();
    return t[0] * 1e3 + t[1] / 1e6;
}

export class BPETrainer {
    constructor(engine, options) {
        this._engine = engine;
        this._vocab = new Vocab();
        this._exact = !!(options && options.exactCompaction);
    }

    get vocab() { return this._vocab; }

    async train(input, options) {
        const opts = options || {};
        const targetVocabSize = opts.targetVocabSize === undefined ? 4096 : opts.targetVocabSize;
        const preTokenizer = opts.preTokenizer || null;
        const onProgress = opts.onProgress || null;
        let bytes = typeof input === 'string' ? new TextEncoder().encode(input) : input;
        let wordStarts = opts.wordStarts || null;
        if (preTokenizer && !wordStarts) {
            // the reference's WASM path (trainer.js:64-80): NFC bytes + word-start mask
            const r = typeof input === 'string' ? preTokenizer.preTokenize(input) : preTokenizer.preTokenizeBytes(bytes);
            if (r.bytes.length > 0 || bytes.length === 0) { bytes = r.bytes; wordStarts = r.wordStarts; }
        }
        if (!bytes || bytes.length === 0) {
            throw new Error('No symbols to train on — corpus is empty after pre-processing');
        }
        const n = native();
        const needed = targetVocabSize - this._vocab.size;
        const trainer = n.trainerCreate(this._engine.device, bytes, wordStarts, {
            targetVocabSize: targetVocabSize,
            vocabSize: this._vocab.size,
            nextTokenId: this._vocab.nextTokenId,
            batchSize: BATCH_SIZE,
            exact: this._exact,
        });
        const merges = [];
        const start = nowMs();
        let done = 0;
        let earlyStop = false;
        try {
            while (done < needed && !earlyStop) {
                const r = await n.trainerStep(trainer, BATCH_SIZE);
                const m = r.merges;
                const k = m.length / 4;
                for (let i = 0; i < k; i++) {
                    const a = m[4 * i];
                    const b = m[4 * i + 1];
                    merges.push([a, b, this._vocab.addMerge(a, b)]);
                }
                done += k;
                earlyStop = r.earlyStop || k === 0;
                const elapsed = (nowMs() - start) / 1000;
                if (onProgress) {
                    onProgress({
                        mergeIndex: done,
                        totalMerges: needed,
                        mergeString: k > 0 ? this._vocab.strings[this._vocab.strings.length - 1] : '—',
                        bestCount: k > 0 ? m[4 * (k - 1) + 3] : 0,
                        symbolCount: r.symbolCount,
                        mergesPerSecond: elapsed > 0 ? done / elapsed : 0,
                    });
                }
            }
        } finally {
            n.trainerDestroy(trainer);
        }
        const total = (nowMs() - start) / 1000;
        return {
            vocab: this._vocab.entries,
            vocabStrings: this._vocab.strings,
            vocabSize: this._vocab.size,
            merges: merges,
            trainingTime: formatDuration(total),
        };
    }

    exportVocab() { return this._vocab.export(); }
}
