"""Vocabulary registry — behaviour of the reference src/bpe/vocab.js.

256 single-byte base tokens; ``add_merge(a, b)`` appends the concatenation
of the two byte strings under the next id (vocab.js:118-124); display
strings follow vocab.js:18-88 and ``export()`` vocab.js:130-143.
"""
from __future__ import annotations


def _hex(b: int) -> str:
    return "<0x%02X>" % b


def _ascii(b: int) -> str:
    if b == 0x20:
        return "▁"
    if b == 0x0A:
        return "\\n"
    return chr(b) if 0x21 <= b <= 0x7E else _hex(b)


def _utf8_at(bs, i: int, n: int):
    if i + n > len(bs):
        return None
    for j in range(1, n):
        if (bs[i + j] & 0xC0) != 0x80:
            return None
    try:
        return bytes(bs[i:i + n]).decode("utf-8")
    except UnicodeDecodeError:
        return None


def display_string(bs) -> str:
    out, i = [], 0
    while i < len(bs):
        b = bs[i]
        if b < 0x80:
            out.append(_ascii(b))
            i += 1
        elif b < 0xC0:
            out.append(_hex(b))
            i += 1
        else:
            n = 2 if b < 0xE0 else (3 if b < 0xF0 else 4)
            s = _utf8_at(bs, i, n)
            if s is None:
                out.append(_hex(b))
                i += 1
            else:
                out.append(s)
                i += n
    return "".join(out)


class Vocab:
    def __init__(self):
        self.entries = [[b] for b in range(256)]
        self.strings = [display_string([b]) for b in range(256)]
        self.next_token_id = 256

    @property
    def size(self) -> int:
        return len(self.entries)

    def add_merge(self, symbol_a: int, symbol_b: int) -> int:
        new_id = self.next_token_id
        self.next_token_id += 1
        merged = self.entries[symbol_a] + self.entries[symbol_b]
        self.entries.append(merged)
        self.strings.append(display_string(merged))
        return new_id

    def export(self) -> str:
        head = ["# GPU BPE Vocabulary (WebGPU Trainer)", "# Total tokens: %d" % len(self.entries), ""]
        body = ["%d\t%s\t[%s]" % (i, self.strings[i], ",".join(map(str, e))) for i, e in enumerate(self.entries)]
        return "\n".join(head + body) + "\n"
