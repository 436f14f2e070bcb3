"""The reference's LogWriter/LogReader test scenarios (src/db/log.rs:282-811), restated as functions
over a reader factory so the same scenarios run against the host LogReader (CPU tests) and the
device-verified BatchLogReader (GPU tests)."""
BLOCK_SIZE, HEADER_SIZE = 32768, 7


def big_string(partial, n):
    s = (partial * (n // len(partial) + 1))[:n]
    return s.encode() if isinstance(s, str) else s


class Tester:
    """LogTest (log.rs:395-508): writer over a memory file, reader created lazily from the bytes."""

    def __init__(self, lcrc, make_reader):
        self.lcrc = lcrc
        self.make_reader = make_reader
        self.writer = lcrc.LogWriter()
        self.prefix = b""
        self.file = None  # mutable copy once reading starts
        self.reader = None
        self.force = False

    def write(self, data):
        assert self.reader is None
        self.writer.add_record(data.encode() if isinstance(data, str) else data)

    def contents(self):
        if self.file is None:
            self.file = bytearray(self.prefix + self.writer.contents())
        return self.file

    def writen_bytes(self):
        return len(self.prefix) + len(self.writer)

    def reopen_for_append(self):
        self.prefix += self.writer.contents()
        self.writer = self.lcrc.LogWriter()  # LogWriter::new(dest) -> offset 0 (log.rs:483-485)

    def _r(self):
        if self.reader is None:
            self.reader = self.make_reader(bytes(self.contents()))
            if self.force:
                self.reader.force_error()
        return self.reader

    def read(self):
        return self._r().read_record()

    def read_string(self):
        return self.read().decode()

    def assert_read_eof(self):
        try:
            self.read()
        except self.lcrc.EofError as e:
            assert str(e) == "meet a eof"
            return
        raise AssertionError("expected eof")

    def dropped_bytes(self):
        return self._r().dropped_bytes

    def report_message(self):
        return self._r().report_message

    def match_error(self, partial):
        return partial in self.report_message()

    def increment_byte(self, off, delta):
        f = self.contents()
        f[off] = (f[off] + delta) & 0xFF

    def set_byte(self, off, b):
        self.contents()[off] = b

    def fix_checksum(self, header_offset, length):
        # log.rs:477-487: crc32fast over file[header_offset+6 .. +len+1], written at offset 0
        f = self.contents()
        c = self.lcrc.value(bytes(f[header_offset + 6:header_offset + 7 + length]))
        f[0:4] = c.to_bytes(4, "little")

    def shrink_size(self, n):
        f = self.contents()
        del f[len(f) - n:]

    def force_error(self):
        self.force = True


def t_read_write(t):
    cases = ["foo", "bar", "abcdefg", "xxxx", "leveldb牛逼", "1234567890", "!@#@#%#$GGTH&FD^^^'fdt'GDDfdfgdfhd21545"]
    for c in cases:
        t.write(c)
    for c in cases:
        assert t.read_string() == c
    t.assert_read_eof()
    t.assert_read_eof()


def t_many_blocks(t, n=1000000):  # log.rs:535-545: 1,000,000 records
    for i in range(n):
        t.write(str(i))
    for i in range(n):
        assert t.read_string() == str(i)
    t.assert_read_eof()


def t_fragment(t):
    cases = [b"small", big_string("medium", 50000), big_string("large", 100000), big_string("larger", 200000)]
    for c in cases:
        t.write(c)
    for c in cases:
        assert t.read() == c
    t.assert_read_eof()


def t_marginal_trailer(t):
    n = BLOCK_SIZE - 2 * HEADER_SIZE
    t.write(big_string("foo", n))
    assert t.writen_bytes() == BLOCK_SIZE - HEADER_SIZE
    t.write(b"\x00")
    t.write("bar")
    assert t.read() == big_string("foo", n)
    assert t.read() == b"\x00"
    assert t.read_string() == "bar"


def t_marginal_trailer2(t):
    n = BLOCK_SIZE - 2 * HEADER_SIZE
    t.write(big_string("foo", n))
    assert t.writen_bytes() == BLOCK_SIZE - HEADER_SIZE
    t.write("bar")
    assert t.read() == big_string("foo", n)
    assert t.read_string() == "bar"
    t.assert_read_eof()
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def t_shorter_trailer(t):
    n = BLOCK_SIZE - 2 * HEADER_SIZE + 4
    t.write(big_string("foo", n))
    assert t.writen_bytes() == BLOCK_SIZE - HEADER_SIZE + 4
    t.write(b"\x00")
    t.write("bar")
    assert t.read() == big_string("foo", n)
    assert t.read() == b"\x00"
    assert t.read_string() == "bar"
    t.assert_read_eof()


def t_aligned_eof(t):
    n = BLOCK_SIZE - 2 * HEADER_SIZE + 4
    t.write(big_string("foo", n))
    assert t.writen_bytes() == BLOCK_SIZE - HEADER_SIZE + 4
    assert t.read() == big_string("foo", n)
    t.assert_read_eof()


def t_open_for_append(t):
    t.write("hello")
    t.reopen_for_append()
    t.write("world")
    assert t.read_string() == "hello"
    assert t.read_string() == "world"
    t.assert_read_eof()


def t_random_read(t, rng):
    strs = []
    for i in range(300):
        high = 1 << int(rng.integers(1, 17))
        n = int(rng.integers(1, high))
        strs.append(big_string(str(i), n))
    for s in strs:
        t.write(s)
    for s in strs:
        assert t.read() == s


def t_read_error(t):
    t.write("foo")
    t.force_error()
    t.assert_read_eof()
    assert t.match_error("read error")


def t_bad_record_type(t):
    t.write("foo")
    t.increment_byte(6, 100)
    t.fix_checksum(0, 3)
    t.assert_read_eof()
    assert t.dropped_bytes() == 3
    assert t.match_error("unknown record type")


def t_truncated_trailing_record_is_ignored(t):
    t.write("foo")
    t.shrink_size(4)
    t.assert_read_eof()
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def t_bad_length(t):
    payload = BLOCK_SIZE - HEADER_SIZE
    t.write(big_string("bar", payload))
    # increment_byte happens on the file; the second write must land after it in the same file
    t.write("foo")
    t.increment_byte(4, 1)
    assert t.read_string() == "foo"
    assert t.dropped_bytes() == BLOCK_SIZE
    assert t.match_error("bad record length")


def t_bad_length_at_end_is_ignored(t):
    t.write("foo")
    t.shrink_size(1)
    t.assert_read_eof()
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def t_checksum_mismatch(t):
    t.write("foo")
    t.increment_byte(0, 10)
    t.assert_read_eof()
    assert t.dropped_bytes() == 10
    assert t.match_error("checksum mismatch")


def t_unexpected_middle_type(t):
    t.write("foo")
    t.set_byte(6, 3)
    t.fix_checksum(0, 3)
    t.assert_read_eof()
    assert t.dropped_bytes() == 3
    assert t.match_error("missing start")


def t_unexpected_last_type(t):
    t.write("foo")
    t.set_byte(6, 4)
    t.fix_checksum(0, 3)
    t.assert_read_eof()
    assert t.dropped_bytes() == 3
    assert t.match_error("missing start")


def t_unexpected_full_type(t):
    t.write("foo")
    t.write("bar")
    t.set_byte(6, 2)
    t.fix_checksum(0, 3)
    assert t.read_string() == "bar"
    t.assert_read_eof()
    assert t.dropped_bytes() == 3
    assert t.match_error("partial record without end")


def t_missing_last_is_ignored(t):
    t.write(big_string("bar", BLOCK_SIZE))
    t.shrink_size(14)
    t.assert_read_eof()
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def t_partial_last_is_ignored(t):
    t.write(big_string("bar", BLOCK_SIZE))
    t.shrink_size(1)
    t.assert_read_eof()
    assert t.dropped_bytes() == 0
    assert t.report_message() == ""


def t_error_joins_record(t):
    t.write(big_string("foo", BLOCK_SIZE))
    t.write(big_string("bar", BLOCK_SIZE))
    t.write("correct")
    for i in range(BLOCK_SIZE, 2 * BLOCK_SIZE):
        t.set_byte(i, ord("x"))
    assert t.read_string() == "correct"
    t.assert_read_eof()
    d = t.dropped_bytes()
    assert 2 * BLOCK_SIZE <= d <= 2 * BLOCK_SIZE + 100


SCENARIOS = [t_read_write, t_fragment, t_marginal_trailer, t_marginal_trailer2, t_shorter_trailer, t_aligned_eof,
             t_open_for_append, t_bad_record_type, t_truncated_trailing_record_is_ignored, t_bad_length,
             t_bad_length_at_end_is_ignored, t_checksum_mismatch, t_unexpected_middle_type, t_unexpected_last_type,
             t_unexpected_full_type, t_missing_last_is_ignored, t_partial_last_is_ignored, t_error_joins_record]
