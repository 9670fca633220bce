"""Test helper: the crate's streaming semantics (stream.rs:77-297) replayed on top of any engine
with search(): WindowReader cuts (64 KiB reads, window growth, valid-UTF-8 prefix, commit at the
overlap-th grapheme from the end via regex \\X), per-window sorted + non-overlapping search,
ownership filter start < commit, absolute offsets."""
import regex

from fuzzy_aho_corasick import SearchOptions as O


def _valid_prefix(buf: bytes) -> int:
    try:
        buf.decode("utf-8")
        return len(buf)
    except UnicodeDecodeError as e:
        return e.start


def stream_rows(engine, data: bytes, threshold: float, overlap: int, window: int = 256 * 1024, chunk=64 * 1024):
    out, buf, base, pos, done = [], b"", 0, 0, False
    while not done:
        while len(buf) < window and pos < len(data):
            buf += data[pos:pos + chunk]
            pos += chunk
        eof = len(buf) < window
        text = buf[:_valid_prefix(buf)].decode("utf-8")
        if eof:
            commit, done = len(text.encode("utf-8")), True
        else:
            starts, off = [], 0
            for g in regex.findall(r"\X", text):
                starts.append(off)
                off += len(g.encode("utf-8"))
            if len(starts) < overlap or starts[len(starts) - overlap] == 0:
                window += max(window, 64 * 1024)
                continue
            commit = starts[len(starts) - overlap]
        for m in engine.search(text, O().threshold(threshold).sorted().non_overlapping()):
            if m.start < commit:
                out.append((base + m.start, base + m.end, m.pattern_index, m.sim_bits(), m.text))
        if not done:
            buf = buf[commit:]
            base += commit
    return out
