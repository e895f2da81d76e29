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


def test_pencil_exact_dispatch_bounds(tsa):
    """pencil_exact: the 12-bit RTL wrap is checked against the bare value
    bound and the carrier against the bound plus a few penalties -- pencil up
    to 680 per side with 12-bit words, exact f16 up to ~676, the literal plane
    kernel beyond (async), the checked lap kernel beyond (synchronous)."""
    for L, want in [(256, "pencil"), (512, "pencil"), (600, "pencil"), (680, "pencil"),
                    (681, "plane"), (1024, "plane")]:
        assert tsa.describe_plan(1, L, L, L, sync=False).split()[0] == want, L
        checked = tsa.describe_plan(1, L, L, L, sync=True).split(" est=")[0].endswith(" checked")
        assert checked == (want == "plane"), L
    assert " f16 " in tsa.describe_plan(1, 512, 512, 512)
    assert " i16 " in tsa.describe_plan(1, 680, 680, 680)


def test_ram128_image_round_trip(tsa, tmp_path):
    """The testbench's sequence RAM (src/TriAlign_tb.sv:94-96,149-169): 32
    four-bit symbols per 128-bit word, symbol i at bits [4(i%32)+3 : 4(i%32)]
    of word i/32 -- packed, as $readmemh text, as raw words."""
    rng = np.random.default_rng(3)
    for n in (1, 31, 32, 33, 64, 100):
        s = rng.integers(0, 5, n).astype(np.uint8)
        w = tsa.pack_ram128(s)
        assert w.shape == ((n + 31) // 32, 16)
        assert np.array_equal(tsa.unpack_ram128(w, n), s)
        # nibble placement: symbol i of word 0 is bits [4i+3:4i] of the 128-bit word
        word0 = int.from_bytes(bytes(w[0]), "little")
        assert all(((word0 >> (4 * i)) & 15) == s[i] for i in range(min(n, 32)))
        hx = tmp_path / f"s{n}.hex"
        hx.write_text("\n".join(tsa.ram128_hex_lines(s)) + "\n")
        assert np.array_equal(tsa.read_sequence(str(hx), "ramhex", n), s)
        raw = tmp_path / f"s{n}.bin"
        w.tofile(str(raw))
        assert np.array_equal(tsa.read_sequence(str(raw), "ramraw", n), s)
    with pytest.raises(tsa.TsaError):
        tsa.unpack_ram128(np.zeros((1, 16), np.uint8), 33)


def test_testbench_initial_block_reader(tsa, orc, tmp_path):
    """The testbench's own input format: `seqA_ram[w][hi:lo] <= SYM;` writes in
    an initial block (src/TriAlign_tb.sv:423-1960). A synthetic block in that
    form round-trips; when the reference tree is present its testbench is read
    directly -- all-A, A_LENGTH = 64 (src/TriAlign_tb.sv:48) -> score 192."""
    rng = np.random.default_rng(4)
    s = rng.integers(0, 5, 70).astype(np.uint8)
    names = "ATCGN"
    lines = [f"seqB_ram[{i // 32}][{4 * (i % 32) + 3}:{4 * (i % 32)}] <= {names[v]};"
             for i, v in enumerate(s)]
    f = tmp_path / "tb.sv"
    f.write_text("initial begin\n" + "\n".join(lines) + "\nend\n")
    assert np.array_equal(tsa.read_sequence(str(f), ram="seqB_ram"), s)
    tb = "/root/reference/src/TriAlign_tb.sv"
    if os.path.exists(tb):
        seqs = [tsa.read_sequence(tb, ram=f"seq{k}_ram", length=64) for k in "ABC"]
        assert all(len(x) == 64 and not x.any() for x in seqs)
        assert orc.score(*seqs) == 192


def test_pack2_layout(tsa):
    """tsa_pack2: four symbols per byte, symbol i at bits 2(i%4); N (4) packs
    as A (the RTL's 2-bit symbol registers, src/PE_1cyc.v:63-66)."""
    rng = np.random.default_rng(12)
    for n in (0, 1, 3, 4, 5, 17, 64, 101):
        s = rng.integers(0, 5, n).astype(np.uint8)
        w = tsa.pack2(s)
        assert len(w) == (n + 3) // 4
        back = np.array([(int(w[i // 4]) >> (2 * (i % 4))) & 3 for i in range(n)], np.uint8)
        assert np.array_equal(back, s & 3)
    with pytest.raises(tsa.TsaError):
        tsa.pack2(np.array([0, 5], np.uint8))
    # int-typed input must not wrap into a valid symbol (256 -> 0 = 'A')
    for bad in (np.array([0, 256], np.int64), np.array([1, -1], np.int32), np.array([0.0, 1.0])):
        with pytest.raises(tsa.TsaError):
            tsa.pack2(bad)
        with pytest.raises(tsa.TsaError):
            tsa.validate(bad, [0], [0])
    assert list(tsa.pack2(np.array([1, 2, 3, 4], np.int64))) == [0b00111001]
