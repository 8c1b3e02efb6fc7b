"""Seeded generators of compressible corpora for the zstd blob stage:
the ratio of the GPU encoder is compared with libzstd level 1 (the reference's
`zstd::stream::copy_encode(data, .., 1)`, pbs-datastore/src/data_blob.rs:151) on data
that looks like what a host backup feeds the chunker.  Nothing is downloaded: every byte
comes from numpy's PCG64 with a fixed seed, so the corpora are identical on every box.

text(n, seed)  English-like prose: a 4096-word vocabulary built from syllables, word
               frequencies Zipf(1.1), sentences of 4-22 words with commas, lines of about
               72 characters, blank lines between paragraphs, some numbers.
pxar(n, seed)  the layout of a pxar archive (the client's host-backup stream,
               pbs-client/src/pxar/create.rs; format of the external `pxar` crate 0.10,
               whose constants are not in the reference tree -- the 64-bit record type
               codes here are placeholders): per file an ENTRY record (16-byte header
               {type, size} + mode, flags, uid, gid, mtime), a FILENAME record, a PAYLOAD
               record with the contents -- text files (prose, config key/value lines,
               C-like source), ELF-like binaries (headers, zero padding, symbol tables of
               increasing offsets, random code bytes), already-compressed files (random
               bytes) -- and per directory a GOODBYE table of {hash, offset, size} items.
"""
import numpy as np

_SYL = ["ba", "be", "bi", "bo", "ca", "ce", "co", "da", "de", "di", "do", "fa", "fe", "fi", "ga",
        "ge", "go", "ha", "he", "hi", "ho", "ja", "ka", "ke", "ki", "la", "le", "li", "lo", "lu",
        "ma", "me", "mi", "mo", "mu", "na", "ne", "ni", "no", "nu", "pa", "pe", "pi", "po", "ra",
        "re", "ri", "ro", "ru", "sa", "se", "si", "so", "ta", "te", "ti", "to", "tu", "va", "ve",
        "vi", "vo", "za", "ze", "an", "en", "in", "on", "ar", "er", "or", "st", "th", "ch", "sh",
        "ck", "nd", "nt", "ll", "ss"]


def _vocab(rng, n=4096):
    words, seen = [], set()
    while len(words) < n:
        k = int(rng.integers(1, 5))
        w = "".join(_SYL[int(i)] for i in rng.integers(0, len(_SYL), k))
        if w not in seen:
            seen.add(w)
            words.append(w)
    p = 1.0 / np.arange(1, n + 1) ** 1.1
    return words, p / p.sum()


def _prose(rng, words, p, nbytes):
    out, size = [], 0
    ids = rng.choice(len(words), size=nbytes // 5 + 64, p=p)
    lens = rng.integers(4, 23, size=ids.size)
    i = j = col = 0
    while size < nbytes:
        n = int(lens[j % lens.size])
        j += 1
        sent = []
        for k in range(n):
            w = words[int(ids[i % ids.size])]
            i += 1
            if k == 0:
                w = w.capitalize()
            if k < n - 1 and rng.random() < 0.08:
                w += ","
            if rng.random() < 0.02:
                w = str(int(rng.integers(0, 100000)))
            sent.append(w)
        s = " ".join(sent) + ". "
        if rng.random() < 0.05:
            s += "\n\n"
            col = 0
        out.append(s)
        col += len(s)
        if col > 72:
            out.append("\n")
            col = 0
        size += len(s) + 1
    return "".join(out).encode()[:nbytes]


def text(n: int, seed: int = 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    words, p = _vocab(rng)
    return np.frombuffer(_prose(rng, words, p, n), dtype=np.uint8).copy()


_T_ENTRY, _T_FILENAME, _T_PAYLOAD, _T_GOODBYE = (0x1396FABCEA5BBB51, 0x16701121063917B3,
                                                  0x28147A1B0B7C1A25, 0x2FEC4FA642D5731D)


def _rec(t, body: bytes) -> bytes:
    return np.array([t, 16 + len(body)], dtype="<u8").tobytes() + body


def _config(rng, words, p, nbytes):
    lines, size = [], 0
    while size < nbytes:
        k = rng.choice(len(words), size=3, p=p)
        v = rng.integers(0, 4)
        val = (str(int(rng.integers(0, 65536))) if v == 0 else "yes" if v == 1 else
               "/usr/lib/" + words[int(k[2])] if v == 2 else words[int(k[2])])
        ln = f"{words[int(k[0])]}_{words[int(k[1])]} = {val}\n"
        if rng.random() < 0.1:
            ln = f"# {words[int(k[1])]} {words[int(k[2])]} {words[int(k[0])]}\n" + ln
        lines.append(ln)
        size += len(ln)
    return "".join(lines).encode()[:nbytes]


def _source(rng, words, p, nbytes):
    out, size, depth = [], 0, 0
    kw = ["if", "for", "while", "return", "int", "static", "const", "struct", "void", "uint64_t"]
    while size < nbytes:
        r = rng.random()
        a, b, c = (words[int(x)] for x in rng.choice(len(words), size=3, p=p))
        if r < 0.1 and depth < 4:
            ln = f"{kw[int(rng.integers(0, 10))]} {a}_{b}({c}) {{"
            depth += 1
        elif r < 0.2 and depth > 0:
            depth -= 1
            ln = "}"
        elif r < 0.3:
            ln = f"/* {a} {b} {c} */"
        else:
            ln = f"{a}->{b} = {c}_{a}({b}, {int(rng.integers(0, 256))});"
        s = "    " * depth + ln + "\n"
        out.append(s)
        size += len(s)
    return "".join(out).encode()[:nbytes]


def _elf(rng, nbytes):
    parts, size = [], 0
    hdr = np.zeros(64, np.uint8)
    hdr[:4] = [0x7F, 0x45, 0x4C, 0x46]
    hdr[4:8] = [2, 1, 1, 0]
    parts.append(hdr.tobytes())
    size += 64
    while size < nbytes:
        r = rng.random()
        if r < 0.35:  # code: random-ish bytes with a skewed opcode distribution
            m = int(rng.integers(256, 8192))
            b = rng.integers(0, 256, m).astype(np.uint8)
            common = np.array([0x48, 0x89, 0x8B, 0xE8, 0x0F, 0x85, 0xC3, 0x00, 0xFF, 0x24], np.uint8)
            sel = rng.random(m) < 0.45
            b[sel] = common[rng.integers(0, common.size, int(sel.sum()))]
            parts.append(b.tobytes())
        elif r < 0.6:  # symbol / relocation tables: increasing offsets, small fields
            m = int(rng.integers(16, 512))
            off = np.cumsum(rng.integers(1, 300, m)).astype("<u8") + 0x400000
            tab = np.zeros((m, 3), dtype="<u8")
            tab[:, 0] = off
            tab[:, 1] = rng.integers(0, 40, m)
            tab[:, 2] = rng.integers(0, 4096, m)
            parts.append(tab.tobytes())
        elif r < 0.8:  # zero padding to an alignment
            parts.append(bytes(int(rng.integers(16, 4096))))
        else:  # string table
            parts.append(b"\0".join(f"_Z{int(rng.integers(1, 30))}sym_{int(rng.integers(0, 5000))}".encode()
                                    for _ in range(int(rng.integers(8, 128)))))
        size += len(parts[-1])
    return b"".join(parts)[:nbytes]


def pxar(n: int, seed: int = 2) -> np.ndarray:
    rng = np.random.default_rng(seed)
    words, p = _vocab(rng)
    exts = [".txt", ".conf", ".c", ".h", ".so", ".gz", ".md", ".py", ""]
    out, size, mtime, items = [], 0, 1_700_000_000, []
    while size < n:
        kind = rng.choice(5, p=[0.3, 0.2, 0.2, 0.15, 0.15])
        flen = int(min(rng.lognormal(8.0, 1.6), 4 << 20))
        name = (words[int(rng.choice(len(words), p=p))] + "_" + words[int(rng.integers(0, len(words)))]
                + exts[int(rng.integers(0, len(exts)))]).encode() + b"\0"
        if kind == 0:
            body = _prose(rng, words, p, flen)
        elif kind == 1:
            body = _config(rng, words, p, flen)
        elif kind == 2:
            body = _source(rng, words, p, flen)
        elif kind == 3:
            body = _elf(rng, flen)
        else:
            body = rng.integers(0, 256, flen, dtype=np.uint8).tobytes()
        mtime += int(rng.integers(0, 5000))
        stat = np.array([0o100644 if kind != 3 else 0o100755, 0], dtype="<u8").tobytes() + \
            np.array([1000, 1000], dtype="<u4").tobytes() + \
            np.array([mtime], dtype="<i8").tobytes() + np.array([int(rng.integers(0, 10**9)), 0], dtype="<u4").tobytes()
        rec = _rec(_T_ENTRY, stat) + _rec(_T_FILENAME, name) + _rec(_T_PAYLOAD, body)
        items.append((int(rng.integers(0, 1 << 63)), size, len(rec)))
        out.append(rec)
        size += len(rec)
        if len(items) >= int(rng.integers(8, 40)):  # close the directory
            gb = np.array(items, dtype="<u8").tobytes()
            out.append(_rec(_T_GOODBYE, gb))
            size += 16 + len(gb)
            items = []
    return np.frombuffer(b"".join(out)[:n], dtype=np.uint8).copy()
