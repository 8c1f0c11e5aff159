// Golden-vector generator for the GPT-4 rule pre-tokenizer: executes the
// REFERENCE's own src/wasm/pre_tokenizer.mjs (read in place from
// /root/reference, never copied) under the container's Node 12.  TEST
// INFRASTRUCTURE ONLY — runs in the dev container to (re)generate
// tests/golden/ref_pretok.json and never travels to the GPU box.
//
// The reference pairs PreTokenizer with its Decoder WASM (Unicode 17 tables),
// which Node 12 cannot compile (SURVEY §8(c)).  The decoder is therefore a
// stand-in built on Node's ICU property escapes (\p{L} \p{M} \p{Nd} \p{N}
// \p{White_Space} \p{P} \p{S}); normalizeBytes is the identity (inputs are
// NFC) and classifyBytes throws, so preTokenizeBytes takes its own JS
// classification fallback (pre_tokenizer.mjs:479-491).  Everything else —
// utf8ToCodepoints, findWordBoundaries, the byte mapping — is the reference's.
//
// usage: node --experimental-vm-modules run_ref_pretok.mjs < cases.json > out.json

import vm from 'vm';
import fs from 'fs';

const REF = process.env.GBPE_REFERENCE || '/root/reference';

const re = {
    L: /^\p{L}$/u, M: /^\p{M}$/u, Nd: /^\p{Nd}$/u, N: /^\p{N}$/u,
    WS: /^\p{White_Space}$/u, P: /^\p{P}$/u, S: /^\p{S}$/u,
};
const t = (r, cp) => r.test(String.fromCodePoint(cp));
const StandInDecoder = {
    isLetter: (cp) => t(re.L, cp),
    isMark: (cp) => t(re.M, cp),
    isDigit: (cp) => t(re.Nd, cp),
    isNumber: (cp) => t(re.N, cp),
    isWhitespace: (cp) => t(re.WS, cp),
    isPunctuation: (cp) => t(re.P, cp),
    isSymbol: (cp) => t(re.S, cp),
    normalize: (s) => s,
    normalizeBytes: (b) => b,
    classifyBytes: () => { throw new Error('stand-in: use the JS classifier'); },
};

async function main() {
    const src = fs.readFileSync(REF + '/src/wasm/pre_tokenizer.mjs', 'utf8');
    const mod = new vm.SourceTextModule(src, { identifier: 'pre_tokenizer.mjs' });
    await mod.link(async (spec) => { throw new Error('unexpected import ' + spec); });
    await mod.evaluate();
    const { PreTokenizer } = mod.namespace;
    console.warn = () => {};
    const pt = new PreTokenizer(StandInDecoder);
    const input = JSON.parse(fs.readFileSync(0, 'utf8'));
    const out = [];
    for (const c of input.cases) {
        const bytes = Uint8Array.from(Buffer.from(c.hex, 'hex'));
        const r = pt.preTokenizeBytes(bytes);
        out.push({ name: c.name, bytes: Buffer.from(r.bytes).toString('hex'),
                   word_starts: Buffer.from(r.wordStarts).toString('hex') });
    }
    process.stdout.write(JSON.stringify({ node: process.version, icu: process.versions.icu,
                                          unicode: process.versions.unicode, cases: out }));
}
main().catch((e) => { console.error(e); process.exit(1); });
