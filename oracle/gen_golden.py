"""Regenerate tests/golden/ref_modules.json — TEST INFRASTRUCTURE ONLY.

Runs in the dev container (needs /root/reference and Node 12).  Builds the
input cases, executes the reference's own CPU-side modules on them with
``oracle/ref_js/run_ref_modules.mjs`` and stores inputs + outputs as a
fixture.  The fixture is data: the reference source never leaves
/root/reference.

    python oracle/gen_golden.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))

import bpe_oracle as O  # noqa: E402
from gpubpe import synth  # noqa: E402


def build_cases() -> dict:
    # merge lists: the SURVEY example, one with duplicate byte strings, and
    # oracle-trained lists on small synthetic corpora (the merge list is just
    # an input to vocab.js / trie.js here; training parity is tested elsewhere)
    sp = 32
    t, h, e = ord("t"), ord("h"), ord("e")
    m_survey = [[t, h], [256, e], [sp, 257]]
    m_dup = [[t, h], [256, e], [h, e], [t, 258]]            # 257 and 259 are both "the"
    en = synth.english(16384, seed=11)
    m_en = [m[:2] for m in O.train(en, 512)["merges"]]
    ml = synth.multilingual(16384, seed=12)
    m_ml = [m[:2] for m in O.train(ml, 400)["merges"]]
    raw = bytes(range(256)) * 4 + b"\x00\x00 \n\n\xff\xfe"
    m_raw = [m[:2] for m in O.train(raw, 300)["merges"]]

    vocab_cases = [
        {"name": "survey_the", "merges": m_survey},
        {"name": "dup_the", "merges": m_dup},
        {"name": "english16k_512", "merges": m_en},
        {"name": "multilingual16k_400", "merges": m_ml},
        {"name": "raw_bytes", "merges": m_raw},
    ]
    trie_cases = []
    for vc in vocab_cases:
        v = O.vocab_from_merges(vc["merges"])
        trie_cases.append({"name": vc["name"], "vocab": v.entries})
    # a vocab with holes (empty entries are skipped by the compiler) and no single bytes
    holes = [[] for _ in range(256)] + [[97, 98], [97, 98, 99], [120]]
    trie_cases.append({"name": "holes_no_bytes", "vocab": holes})

    texts = ["the then the", "There is the thing, then the other thing.\n", "aaaa aaa",
             en[:2000].decode("latin-1"), ml[:1500].decode("utf-8", "ignore")]
    merge_encode_cases = []
    for vc in vocab_cases:
        v = O.vocab_from_merges(vc["merges"])
        merges = [[a, b, 256 + i] for i, (a, b) in enumerate(vc["merges"])]
        model = {"vocab": v.entries, "merges": merges}
        for k, tx in enumerate(texts):
            merge_encode_cases.append({"name": f"{vc['name']}#{k}", "model": model, "text": tx})
    return {"vocab_cases": vocab_cases, "trie_cases": trie_cases,
            "merge_encode_cases": merge_encode_cases}


def main():
    cases = build_cases()
    script = os.path.join(HERE, "ref_js", "run_ref_modules.mjs")
    r = subprocess.run(["node", "--experimental-vm-modules", script], input=json.dumps(cases).encode(),
                       capture_output=True, check=True)
    out = json.loads(r.stdout)
    fixture = {
        "_about": "inputs and outputs of the reference's vocab.js / trie.js / tokenizer-manager.js, "
                  "executed under Node 12 by oracle/ref_js/run_ref_modules.mjs (oracle/gen_golden.py)",
        "inputs": cases, "outputs": out,
    }
    dst = os.path.join(ROOT, "tests", "golden", "ref_modules.json")
    with open(dst, "w") as f:
        json.dump(fixture, f, separators=(",", ":"))
    print("wrote", dst, os.path.getsize(dst), "bytes")


if __name__ == "__main__":
    main()
