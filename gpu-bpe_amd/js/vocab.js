/**
 * Vocab — token registry (behaviour of the reference src/bpe/vocab.js):
 * 256 byte tokens, addMerge(a, b) appends the concatenated byte string
 * under nextTokenId++, display strings (▁ for space, \n, <0xHH> for
 * non-printable / invalid UTF-8), export() text format.
 */
const decoder = new TextDecoder('utf-8', { fatal: true });

function hexByte(b) {
    return '<0x' + b.toString(16).toUpperCase().padStart(2, '0') + '>';
}

function asciiByte(b) {
    if (b === 0x20) return '▁';
    if (b === 0x0A) return '\\n';
    return (b >= 0x21 && b <= 0x7E) ? String.fromCharCode(b) : hexByte(b);
}

function utf8At(bytes, i, len) {
    if (i + len > bytes.length) return null;
    for (let j = 1; j < len; j++) {
        if ((bytes[i + j] & 0xC0) !== 0x80) return null;
    }
    try {
        return decoder.decode(new Uint8Array(bytes.slice(i, i + len)));
    } catch (e) {
        return null;
    }
}

export function displayString(bytes) {
    let out = '';
    let i = 0;
    while (i < bytes.length) {
        const b = bytes[i];
        if (b < 0x80) { out += asciiByte(b); i += 1; continue; }
        if (b < 0xC0) { out += hexByte(b); i += 1; continue; }
        const len = b < 0xE0 ? 2 : (b < 0xF0 ? 3 : 4);
        const s = utf8At(bytes, i, len);
        if (s === null) { out += hexByte(b); i += 1; } else { out += s; i += len; }
    }
    return out;
}

export class Vocab {
    constructor() {
        this.entries = [];
        this.strings = [];
        this.nextTokenId = 256;
        for (let b = 0; b < 256; b++) {
            this.entries.push([b]);
            this.strings.push(displayString([b]));
        }
    }

    get size() { return this.entries.length; }

    addMerge(symbolA, symbolB) {
        const id = this.nextTokenId;
        this.nextTokenId += 1;
        const merged = this.entries[symbolA].concat(this.entries[symbolB]);
        this.entries.push(merged);
        this.strings.push(displayString(merged));
        return id;
    }

    export() {
        const lines = ['# GPU BPE Vocabulary (WebGPU Trainer)', '# Total tokens: ' + this.entries.length, ''];
        for (let i = 0; i < this.entries.length; i++) {
            lines.push(i + '\t' + this.strings[i] + '\t[' + this.entries[i].join(',') + ']');
        }
        return lines.join('\n') + '\n';
    }
}
