"""Host-side logic of the package: input formats, batch packing, the RTL
envelope tag and the TriAlign mirror. No GPU."""
import os

import numpy as np
import pytest


def test_read_dat_crlf(tsa, tmp_path):
    p = tmp_path / "s.dat"
    p.write_bytes(b"3\r\n2\r\n0\r\n4\r\n")
    assert list(tsa.read_sequence(str(p))) == [3, 2, 0, 4]


def test_read_reference_dat_files(tsa, golden):
    d = "/root/reference/dat"
    if not os.path.isdir(d):
        pytest.skip("reference not mounted")
    by = {c["name"]: c for c in golden}
    for f, k in (("A_seq.dat", "a"), ("B_seq.dat", "b"), ("C_seq.dat", "c")):
        assert list(tsa.read_sequence(os.path.join(d, f))) == by["dat"][k]


def test_read_fasta(tsa, tmp_path):
    p = tmp_path / "s.fa"
    p.write_text(">x desc\nACGT\nnu\n>second\nGGG\n")
    assert list(tsa.read_sequence(str(p))) == [0, 2, 3, 1, 4, 1]
    bad = tmp_path / "b.fa"
    bad.write_text(">x\nACXT\n")
    with pytest.raises(tsa.TsaError):
        tsa.read_sequence(str(bad))


def test_string_symbols(tsa):
    assert list(tsa._as_u8("ATCGN")) == [0, 1, 2, 3, 4]


def test_pack_batch(tsa):
    seqs, offs = tsa.pack_batch([([0, 1], [2], [3, 3, 3]), ("AC", "G", "T")])
    assert list(offs) == [0, 2, 3, 6, 8, 9, 10]
    assert list(seqs) == [0, 1, 2, 3, 3, 3, 0, 2, 3, 1]


def test_rtl_envelope(tsa):
    assert tsa.rtl_envelope(64, 64, 64)
    assert tsa.rtl_envelope(512, 256, 512)
    assert not tsa.rtl_envelope(63, 64, 64)     # not a multiple of PE_LEN
    assert not tsa.rtl_envelope(64, 128, 64)    # LB > LA overwrites the corner slot
    assert not tsa.rtl_envelope(1024, 64, 64)   # deeper than the SRAM
    t = tsa.TriAlign()
    assert t.in_envelope(64, 64, 64) and not t.in_envelope(60, 64, 64)


def test_trialign_mirror_display(tsa):
    t = tsa.TriAlign(A_TOTAL_LEN=512, SCORE_BITS=12)
    t.Score = 1
    assert t.display() == "TriAlign Score:        \t1"
    assert t.params.score_bits == 12


def test_synth_batch_layout(synth):
    seqs, offs = synth.batch(3, 4, 10, 12, 14)
    assert len(offs) == 13 and offs[-1] == len(seqs) == 4 * 36
    a, b, c = synth.triple(4, 10, 12, 14)
    assert np.array_equal(seqs[offs[3]:offs[4]], a)
    assert np.array_equal(seqs[offs[5]:offs[6]], c)
