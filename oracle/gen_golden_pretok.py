"""Regenerate tests/golden/ref_pretok.json — TEST INFRASTRUCTURE ONLY.

Runs in the dev container (needs /root/reference and Node 12): executes the
reference's pre_tokenizer.mjs through oracle/ref_js/run_ref_pretok.mjs on the
cases below and stores inputs + outputs (data only).

    python oracle/gen_golden_pretok.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))

from gpubpe import synth  # noqa: E402

CASES = {
    "contractions": "I don't know. They'll say we're sure it's HIS'S, she'd've I'M O'Neil's dogs' 'tis rock'n'roll",
    "curly_apostrophe": "don’t we’re it’s can’T you’LL",
    "digits": "1 12 123 1234 12345 123456 1234567 x1234y 3.14159 1,000,000 2024-10-15 ٣٤٥٦٧ ½¾ 10²",
    "code": "def f(x, y=10):\n    return x**2 + y  # comment's\n\tif (a>=b && c!=d) { z[i] = 0x1F; }\r\n",
    "whitespace": "a  b\t\tc  d　e f\n\n g\r\nh i j\u0085k",
    "punct_runs": "wait... what?!?! (yes) [no] {maybe} <tag/> --flag ==> ::= @@ ## $$$ %%% ^^^ &&& ***",
    "multilingual": "İstanbul'da güzel bir gün. Привет, мир! 你好，世界。مرحبا بالعالم. Ελληνικά κείμενα. हिन्दी पाठ",
    "emoji_symbols": "smile 😀😀 ok 👍🏽 ♥♦ ©®™ € £ ¥ → ← ∑∫√ ±×÷",
    "marks": "é ñ café äb",
    "edge_start": "'s",
    "edge_apostrophe_end": "dogs'",
    "single": "x",
}


def build_cases():
    cases = [{"name": k, "hex": v.encode("utf-8").hex()} for k, v in CASES.items()]
    cases.append({"name": "synth_code_20k", "hex": synth.code(20000, seed=31).hex()})
    cases.append({"name": "synth_multilingual_20k", "hex": synth.multilingual(20000, seed=32).hex()})
    cases.append({"name": "synth_english_20k", "hex": synth.english(20000, seed=33).hex()})
    return cases


def main():
    cases = build_cases()
    r = subprocess.run(["node", "--experimental-vm-modules", os.path.join(HERE, "ref_js", "run_ref_pretok.mjs")],
                       input=json.dumps({"cases": cases}), capture_output=True, text=True, check=True)
    out = json.loads(r.stdout)
    doc = {"_about": "inputs and outputs of the reference's src/wasm/pre_tokenizer.mjs (preTokenizeBytes), executed "
                     "under Node 12 with an ICU stand-in for the Decoder WASM by oracle/ref_js/run_ref_pretok.mjs "
                     "(oracle/gen_golden_pretok.py)",
           "node": out["node"], "icu": out["icu"], "unicode": out["unicode"],
           "inputs": cases, "outputs": out["cases"]}
    path = os.path.join(ROOT, "tests", "golden", "ref_pretok.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=0)
    print(f"{path}: {len(cases)} cases")


if __name__ == "__main__":
    main()
