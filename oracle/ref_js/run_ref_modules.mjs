// Golden-vector generator: executes the REFERENCE's own CPU-side modules
// (read in place from /root/reference, never copied) under the container's
// Node 12 and prints their outputs as JSON.  TEST INFRASTRUCTURE ONLY — it
// runs in the dev container to (re)generate tests/golden/ref_modules.json and
// never travels to, or runs on, the GPU box.
//
// Modules exercised:
//   src/bpe/vocab.js                      Vocab.addMerge / export / strings
//   src/bpe/tokenizer/trie.js             compileVocabToTrie / parseHeader / parseTrieBuffers
//   src/bpe/tokenizer/tokenizer-manager.js TokenizerManager.encode (CPU merge-order encoder)
//
// trie.js imports INVALID_TOKEN from ../engine.js, which Node 12 cannot parse
// (engine.js:76 uses `?.` / `??`).  That single import is linked to a
// synthetic module exporting the same constant (engine.js:12, 0xFFFFFFFF);
// no other reference code is replaced.
//
// usage: node --experimental-vm-modules run_ref_modules.mjs < cases.json > out.json

import vm from 'vm';
import fs from 'fs';

const REF = process.env.GBPE_REFERENCE || '/root/reference';

async function loadModule(path, links) {
    const src = fs.readFileSync(path, 'utf8');
    const mod = new vm.SourceTextModule(src, { identifier: path });
    await mod.link(async (spec) => {
        if (links && links[spec]) return links[spec]();
        throw new Error('unlinked import ' + spec + ' in ' + path);
    });
    await mod.evaluate();
    return mod.namespace;
}

function engineConstants() {
    const m = new vm.SyntheticModule(['INVALID_TOKEN'], function () {
        this.setExport('INVALID_TOKEN', 0xFFFFFFFF);
    });
    return m;
}

function toHex(buf) {
    return Buffer.from(new Uint8Array(buf)).toString('hex');
}

async function main() {
    const input = JSON.parse(fs.readFileSync(0, 'utf8'));
    const { Vocab } = await loadModule(REF + '/src/bpe/vocab.js');
    const trieMod = await loadModule(REF + '/src/bpe/tokenizer/trie.js', { '../engine.js': engineConstants });
    const { TokenizerManager } = await loadModule(REF + '/src/bpe/tokenizer/tokenizer-manager.js');

    const out = { vocab_cases: [], trie_cases: [], merge_encode_cases: [] };

    for (const c of input.vocab_cases) {
        const v = new Vocab();
        const ids = c.merges.map(([a, b]) => v.addMerge(a, b));
        out.vocab_cases.push({
            name: c.name, ids, entries: v.entries, strings: v.strings,
            size: v.size, nextTokenId: v.nextTokenId, export: v.export(),
        });
    }

    for (const c of input.trie_cases) {
        const buf = trieMod.compileVocabToTrie(c.vocab);
        const header = trieMod.parseHeader(buf);
        const { nodes, edges } = trieMod.parseTrieBuffers(buf, header);
        out.trie_cases.push({
            name: c.name, trie_hex: toHex(buf), header,
            nodes: Array.from(nodes), edges: Array.from(edges),
        });
    }

    for (const c of input.merge_encode_cases) {
        const tm = new TokenizerManager(null, { getTrainedModel: () => c.model }, null);
        const r = await tm.encode(c.text);
        out.merge_encode_cases.push({ name: c.name, tokens: r.tokens });
    }

    process.stdout.write(JSON.stringify(out));
}

main().catch((e) => { console.error(e && e.stack || e); process.exit(1); });
