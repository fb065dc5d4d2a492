"""Known-answer tests for the oracle's table functions.

The expected values are worked by hand from the reference tables
(WordsUtils.cs:33-66) and formulas:
  exp2s          WordsUtils.cs:633-646   value = (exp2_table[log & 0xff] | 0x100) shifted by (log >> 8) - 9
  mylog2         WordsUtils.cs:588-608   (bits << 8) + log2_table[next 8 mantissa bits]
  count_bits     WordsUtils.cs:513-537   bit length
  restore_weight WordsUtils.cs:614-626   w << 3, plus (w + 64) >> 7 when positive
  read_code      WordsUtils.cs:546-570   truncated binary code over [0, maxcode], LSB-first bits
"""
import pytest

from oracle import oracle as O


@pytest.mark.parametrize("log,val", [
    (0, 0), (0x100, 1), (0x200, 2), (0x800, 128), (0x900, 256), (0xA00, 512),
    (0x980, 362),              # 2^9.5 = 362.04 -> exp2_table[0x80] = 0x6a
    (-0x100, -1), (-0x900, -256), (0x1100, 65536),
])
def test_exp2s(log, val):
    assert O.lib().wvo_exp2s(log) == val


@pytest.mark.parametrize("x,val", [
    (0, 0), (1, 256), (2, 512), (256, 9 << 8),
    (255, (8 << 8) + 0xff),    # 255 -> mantissa index (255 << 1) & 0xff = 254: log2_table[254] = 0xff
    (3, (2 << 8) + 0x96),      # 3 -> index (3 << 7) & 0xff = 128: log2_table[128] = 0x96 (log2(1.5) * 256)
])
def test_mylog2(x, val):
    assert O.lib().wvo_mylog2(x) == val


@pytest.mark.parametrize("v,bits", [(0, 0), (1, 1), (2, 2), (255, 8), (256, 9), (65535, 16), (2**31 - 1, 31)])
def test_count_bits(v, bits):
    assert O.lib().wvo_count_bits(v) == bits


@pytest.mark.parametrize("w,val", [(0, 0), (1, 8), (64, 516), (127, 1024), (-1, -8), (-128, -1024)])
def test_restore_weight(w, val):
    assert O.lib().wvo_restore_weight(w) == val


@pytest.mark.parametrize("buf,maxcode,code,used", [
    (b"\x00", 0, 0, 0),          # maxcode 0: nothing read
    (b"\x00", 1, 0, 1),          # bitcount 1, extras 0: one extra bit
    (b"\x01", 1, 1, 1),
    (b"\x00", 2, 0, 1),          # bitcount 2, extras 1: code 0 takes one bit
    (b"\x01", 2, 1, 2),          # 1 >= extras -> 2*1-1 + next bit(0)
    (b"\x03", 2, 2, 2),          # ... + next bit(1)
    (b"\x05", 4, 1, 2),          # bitcount 3, extras 3: getbits(2) = 0b01 = 1 < 3 -> code 1
    (b"\x07", 4, 4, 3),          # getbits(2) = 3 >= 3 -> 2*3-3 + next bit(1) = 4
])
def test_read_code(buf, maxcode, code, used):
    assert O.read_code(buf, maxcode) == (code, used)
