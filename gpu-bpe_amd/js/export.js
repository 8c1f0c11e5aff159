/**
 * Model JSON and DXFT export — the reference's training-manager.js:173-224
 * (downloadModel / loadFromJSON, minus the browser download) and
 * export-controller.js:191-248 (.bin v2), for Node.  Node 12 syntax.
 */
const DXFT_MAGIC = 0x44584654; // 'DXFT'

export function modelToJSON(model) {
    return JSON.stringify({ version: 1, vocabSize: model.vocabSize, vocab: model.vocab, merges: model.merges });
}

export function loadModelJSON(jsonData) {
    const obj = typeof jsonData === 'string' ? JSON.parse(jsonData) : jsonData;
    if (!obj.vocab || !obj.merges) throw new Error('Invalid vocabulary file: missing vocab or merges');
    const vocab = obj.vocab;
    const vocabStrings = vocab.map(function (bytes) {
        if (!bytes || bytes.length === 0) return '';
        return Buffer.from(Uint8Array.from(bytes)).toString('utf8');
    });
    return { vocab: vocab, vocabStrings: vocabStrings, vocabSize: vocab.length, merges: obj.merges };
}

/** [MAGIC, vocabSize, tokenCount, vocabBytesLen, ...tokens] + vocab JSON bytes (export-controller.js:234-247) */
export function dxftBin(tokens, vocabSize, vocabExport) {
    const vocabBytes = vocabExport ? Buffer.from(JSON.stringify(vocabExport), 'utf8') : Buffer.alloc(0);
    const out = new Uint32Array(4 + tokens.length);
    out[0] = DXFT_MAGIC;
    out[1] = vocabSize;
    out[2] = tokens.length;
    out[3] = vocabBytes.length;
    out.set(tokens, 4);
    const tokenPart = new Uint8Array(out.buffer);
    const finalBuf = new Uint8Array(tokenPart.length + vocabBytes.length);
    finalBuf.set(tokenPart);
    finalBuf.set(vocabBytes, tokenPart.length);
    return finalBuf;
}

/** export-controller.js:191-248: files joined with "\n\n", GPU trie encode, .bin */
export async function exportDXFT(trieTokenizer, files, vocabExport, model) {
    const sep = Buffer.from('\n\n', 'utf8');
    const parts = [];
    files.forEach(function (f, i) { if (i > 0) parts.push(sep); parts.push(Buffer.from(f)); });
    const merged = new Uint8Array(Buffer.concat(parts));
    const tokens = await trieTokenizer.encodeBytes(merged);
    const exp = vocabExport || (model ? { version: 1, vocabSize: model.vocabSize, vocab: model.vocab,
        merges: model.merges } : null);
    const vocabSize = (vocabExport && vocabExport.vocab && vocabExport.vocab.length) ||
        (model && model.vocabSize) || 256;
    return dxftBin(tokens, vocabSize, exp);
}
