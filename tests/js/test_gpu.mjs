// GPU checks through the N-API addon: BPETrainer / TrieTokenizer results
// must equal the expectations the CPU oracle produced (argv[2] JSON).
import fs from 'fs';
import { BPEEngine, BPETrainer, TrieTokenizer, GpuPreTokenizer, MergeEncoder } from '../../gpu-bpe_amd/js/index.js';

const cases = JSON.parse(fs.readFileSync(process.argv[2]));
function fail(msg) { console.error('FAIL ' + msg); process.exit(1); }

async function main() {
    const engine = await new BPEEngine().init();
    if (Object.keys(engine.pipelines).length < 5) fail('pipelines');
    if (!(engine.limits.maxBufferSize > 0)) fail('limits');
    let checks = 0;
    for (const c of cases.train) {
        const t = new BPETrainer(engine);
        const bytes = new Uint8Array(Buffer.from(c.b64, 'base64'));
        let progress = 0;
        const r = await t.train(bytes, { targetVocabSize: c.target, onProgress: function (p) { progress++; } });
        if (JSON.stringify(r.merges) !== JSON.stringify(c.merges)) fail('merges ' + c.name);
        if (r.vocabSize !== 256 + c.merges.length) fail('vocabSize ' + c.name);
        if (c.merges.length && progress === 0) fail('progress ' + c.name);
        if (t.exportVocab() !== c.export) fail('export ' + c.name);
        checks++;
        const tok = TrieTokenizer.fromVocab(engine, r.vocab, c.chunkSize ? { chunkSize: c.chunkSize } : {});
        const text = new Uint8Array(Buffer.from(c.text_b64, 'base64'));
        const ids = await tok.encodeBytes(text);
        if (JSON.stringify(Array.from(ids)) !== JSON.stringify(c.tokens)) fail('tokens ' + c.name);
        if (Buffer.compare(Buffer.from(tok.decode(ids)), Buffer.from(text)) !== 0) fail('decode ' + c.name);
        tok.destroy();
        checks++;
    }
    if (cases.pretok) {   // GPT-4 rule word starts + training through the preTokenizer option
        const p = cases.pretok;
        const bytes = new Uint8Array(Buffer.from(p.b64, 'base64'));
        const pt = new GpuPreTokenizer(engine);
        const r = pt.preTokenizeBytes(bytes);
        if (JSON.stringify(Array.from(r.wordStarts)) !== JSON.stringify(p.word_starts)) fail('pretok wordStarts');
        const t = await new BPETrainer(engine).train(bytes, { targetVocabSize: p.target, preTokenizer: pt });
        if (JSON.stringify(t.merges) !== JSON.stringify(p.merges)) fail('pretok merges');
        checks += 2;
    }
    if (cases.merge_encode) {   // TokenizerManager.encode semantics on the GPU
        const c = cases.merge_encode;
        const enc = new MergeEncoder(engine, { vocab: [], vocabStrings: [], merges: c.merges });
        const r = await enc.encode(c.text);
        if (JSON.stringify(r.tokens) !== JSON.stringify(c.tokens)) fail('merge encode');
        checks++;
    }
    let threw = false;
    try { await new BPETrainer(engine).train(new Uint8Array(0)); } catch (e) { threw = /empty/.test(e.message); }
    if (!threw) fail('empty corpus must throw');
    {   // concurrency + lifetimes on one engine (the addon serialises a context's device work)
        const c = cases.train[0];
        const r = await new BPETrainer(engine).train(new Uint8Array(Buffer.from(c.b64, 'base64')),
                                                    { targetVocabSize: c.target });
        const tok = TrieTokenizer.fromVocab(engine, r.vocab, c.chunkSize ? { chunkSize: c.chunkSize } : {});
        const text = new Uint8Array(Buffer.from(c.text_b64, 'base64'));
        const all = await Promise.all([tok.encodeBytes(text), tok.encodeBytes(text), tok.encodeBytes(text.subarray(7))]);
        if (JSON.stringify(Array.from(all[0])) !== JSON.stringify(c.tokens)) fail('concurrent encode 0');
        if (JSON.stringify(Array.from(all[1])) !== JSON.stringify(c.tokens)) fail('concurrent encode 1');
        const solo = await tok.encodeBytes(text.subarray(7));
        if (JSON.stringify(Array.from(all[2])) !== JSON.stringify(Array.from(solo))) fail('concurrent encode 2');
        // free the trie while an encode is in flight, then destroy the engine while a
        // training step is in flight: both complete, nothing is used after free
        const n = (await import('../../gpu-bpe_amd/js/native.js')).native();
        const pending = tok.encodeBytes(text);
        tok.destroy();
        const late = await pending;
        if (JSON.stringify(Array.from(late)) !== JSON.stringify(c.tokens)) fail('encode across trie free');
        const e2 = await new BPEEngine().init();
        const tr = n.trainerCreate(e2.device, new Uint8Array(Buffer.from(c.b64, 'base64')), null,
                                   { targetVocabSize: c.target });
        const step = n.trainerStep(tr, 128);
        e2.destroy();
        n.trainerDestroy(tr);
        const s = await step;
        if (s.merges.length !== 4 * Math.min(128, c.merges.length)) fail('step across destroy');
        checks += 4;
    }
    engine.destroy();
    console.log('ok ' + checks + ' checks');
}
main().catch(function (e) { fail(e && e.stack || e); });
