// CPU-only checks of the JS host modules against the reference's own
// vocab.js / trie.js outputs (tests/golden/ref_modules.json).
import fs from 'fs';
import { Vocab, compileVocabToTrie, parseHeader, parseTrieBuffers, dxftBin, modelToJSON, loadModelJSON } from '../../gpu-bpe_amd/js/index.js';

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
// .bin v2 writer == the oracle's restatement of export-controller.js:221-248
{
    const ve = { version: 1, vocabSize: 258, vocab: [[104], [105], [104, 105]], merges: [[104, 105, 257]] };
    const got = Buffer.from(dxftBin(Uint32Array.from([1, 2, 257]), 258, ve)).toString('hex');
    const exp = '544658440201000003000000560000000100000002000000010100007b2276657273696f6e223a312c22766f63616253697a65223a3235382c22766f636162223a5b5b3130345d2c5b3130355d2c5b3130342c3130355d5d2c226d6572676573223a5b5b3130342c3130352c3235375d5d7d';
    if (got !== exp) { console.error('FAIL dxftBin'); process.exit(1); }
    const m = loadModelJSON(modelToJSON({ vocabSize: 3, vocab: ve.vocab, merges: ve.merges }));
    if (m.vocabSize !== 3 || m.vocabStrings[2] !== 'hi') { console.error('FAIL model json'); process.exit(1); }
}
console.log('ok ' + checks + ' checks');
