/**
 * Trie compile / parse — behaviour of the reference src/bpe/tokenizer/trie.js.
 * v3 binary: 28-byte header [TRIE, 3, nodeCount, edgeCount, maxTokenLen,
 * vocabSize, 0], 12-byte nodes {firstChild, numChildren, tokenId}, 8-byte
 * edges {u8 symbol + 3 pad, target}.  BFS order, children by ascending byte,
 * a later duplicate byte string overwrites the token id.  v2 parses too.
 */
import { INVALID_TOKEN } from './engine.js';

const MAGIC = 0x54524945;
const HEADER = 28;

export function compileVocabToTrie(vocab) {
    const root = { kids: new Map(), tid: INVALID_TOKEN };
    let maxLen = 0;
    for (let id = 0; id < vocab.length; id++) {
        const seq = vocab[id];
        if (!seq || seq.length === 0) continue;
        let node = root;
        for (let k = 0; k < seq.length; k++) {
            let nxt = node.kids.get(seq[k]);
            if (!nxt) { nxt = { kids: new Map(), tid: INVALID_TOKEN }; node.kids.set(seq[k], nxt); }
            node = nxt;
        }
        node.tid = id;
        if (seq.length > maxLen) maxLen = seq.length;
    }
    const nodes = [];   // flat [firstChild, numChildren, tokenId]*
    const edges = [];   // flat [symbol, target]*
    const order = [root];
    let nextIndex = 1;
    for (let head = 0; head < order.length; head++) {
        const node = order[head];
        const syms = Array.from(node.kids.keys()).sort(function (x, y) { return x - y; });
        nodes.push(edges.length / 2, syms.length, node.tid);
        for (const s of syms) {
            edges.push(s, nextIndex++);
            order.push(node.kids.get(s));
        }
    }
    const nodeCount = nodes.length / 3;
    const edgeCount = edges.length / 2;
    const buf = new ArrayBuffer(HEADER + nodeCount * 12 + edgeCount * 8);
    const view = new DataView(buf);
    const head = [MAGIC, 3, nodeCount, edgeCount, maxLen, vocab.length, 0];
    for (let i = 0; i < 7; i++) view.setUint32(4 * i, head[i], true);
    let off = HEADER;
    for (let i = 0; i < nodes.length; i++, off += 4) view.setUint32(off, nodes[i] >>> 0, true);
    for (let e = 0; e < edgeCount; e++, off += 8) {
        view.setUint32(off, edges[2 * e] & 0xFF, true);
        view.setUint32(off + 4, edges[2 * e + 1], true);
    }
    return buf;
}

export function parseHeader(data) {
    const view = new DataView(data, 0, HEADER);
    const magic = view.getUint32(0, true);
    const version = view.getUint32(4, true);
    if (magic !== MAGIC) throw new Error('Invalid trie magic: 0x' + magic.toString(16));
    if (version !== 2 && version !== 3) throw new Error('Unsupported trie version: ' + version);
    return {
        version: version,
        nodeCount: view.getUint32(8, true),
        edgeCount: view.getUint32(12, true),
        maxTokenLen: view.getUint32(16, true),
    };
}

export function parseTrieBuffers(data, header) {
    const v3 = header.version === 3;
    const perNode = v3 ? 12 : 8;
    const perEdge = v3 ? 8 : 4;
    const nc = header.nodeCount;
    const ec = header.edgeCount;
    if (data.byteLength < HEADER + nc * perNode + ec * perEdge) throw new Error('Truncated trie data');
    const view = new DataView(data);
    const nodes = new Uint32Array(nc * 3);
    const edges = new Uint32Array(ec * 2);
    let off = HEADER;
    for (let i = 0; i < nc; i++, off += perNode) {
        if (v3) {
            nodes[3 * i] = view.getUint32(off, true);
            nodes[3 * i + 1] = view.getUint32(off + 4, true);
            nodes[3 * i + 2] = view.getUint32(off + 8, true);
        } else {
            nodes[3 * i] = view.getUint16(off, true);
            nodes[3 * i + 1] = view.getUint16(off + 2, true);
            const t = view.getUint16(off + 4, true);
            nodes[3 * i + 2] = t === 0xFFFF ? INVALID_TOKEN : t;
        }
    }
    for (let e = 0; e < ec; e++, off += perEdge) {
        if (v3) {
            edges[2 * e] = view.getUint8(off);
            edges[2 * e + 1] = view.getUint32(off + 4, true);
        } else {
            edges[2 * e] = view.getUint16(off, true) & 0xFF;
            edges[2 * e + 1] = view.getUint16(off + 2, true);
        }
    }
    return { nodes: nodes, edges: edges };
}
