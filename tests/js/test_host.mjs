// CPU-only checks of the JS host modules against the reference's own
// vocab.js / trie.js outputs (tests/golden/ref_modules.json).
import fs from 'fs';
import { Vocab, compileVocabToTrie, parseHeader, parseTrieBuffers } from '../../gpu-bpe_amd/js/index.js';

const golden = JSON.parse(fs.readFileSync(new URL('../golden/ref_modules.json', import.meta.url)));
let checks = 0;
function eq(a, b, what) {
    const sa = JSON.stringify(a), sb = JSON.stringify(b);
    if (sa !== sb) { console.error('MISMATCH ' + what + '\n  got  ' + sa.slice(0, 200) + '\n  want ' + sb.slice(0, 200)); process.exit(1); }
    checks++;
}
const vin = golden.inputs.vocab_cases, vout = golden.outputs.vocab_cases;
for (let i = 0; i < vin.length; i++) {
    const v = new Vocab();
    const ids = vin[i].merges.map(function (m) { return v.addMerge(m[0], m[1]); });
    eq(ids, vout[i].ids, 'ids ' + vin[i].name);
    eq(v.entries, vout[i].entries, 'entries ' + vin[i].name);
    eq(v.strings, vout[i].strings, 'strings ' + vin[i].name);
    eq(v.export(), vout[i].export, 'export ' + vin[i].name);
}
const tin = golden.inputs.trie_cases, tout = golden.outputs.trie_cases;
for (let i = 0; i < tin.length; i++) {
    const buf = compileVocabToTrie(tin[i].vocab);
    eq(Buffer.from(new Uint8Array(buf)).toString('hex'), tout[i].trie_hex, 'trie ' + tin[i].name);
    const h = parseHeader(buf);
    eq(h, tout[i].header, 'header ' + tin[i].name);
    const b = parseTrieBuffers(buf, h);
    eq(Array.from(b.nodes), tout[i].nodes, 'nodes ' + tin[i].name);
    eq(Array.from(b.edges), tout[i].edges, 'edges ' + tin[i].name);
}
console.log('ok ' + checks + ' checks');
