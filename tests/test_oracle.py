"""Pin the C restatement oracle (oracle/srtp_oracle.c) before trusting it.

Two independent anchors:
  * the reference's own known-answer tests, transcribed as data from
    test/srtp.c, test/aes.c, test/hmac.c and test/sha.c;
  * tests/golden/srtp_golden.json.gz, produced by the reference itself
    (oracle/gen_golden.c linked against /root/reference sources + OpenSSL).
CPU only.
"""
import pytest

from tests import oracle_lib as O
from tests.golden_util import replay_scenario

H = bytes.fromhex


# test/srtp.c:81-133 -- RFC 3711 B.2 AES-CM keystream
def test_rfc3711_b2_keystream():
    ks = O.aes_ctr(H("2B7E151628AED2A6ABF7158809CF4F3C"),
                   H("F0F1F2F3F4F5F6F7F8F9FAFBFCFD0000"), bytes(48))
    assert ks == H("E03EAD0935C95E80E166B16DD92B4EB4"
                   "D23513162B02D0F72A43A2FE4A5F97AB"
                   "41E95B3BB0A2E8DD477901E4FCA894C0")


# test/srtp.c:139-194 -- RFC 6188 7.1 AES-256-CM keystream
def test_rfc6188_keystream():
    ks = O.aes_ctr(H("57f82fe3613fd170a85ec93c40b1f092"
                     "2ec4cb0dc025b58272147cc438944a98"),
                   H("F0F1F2F3F4F5F6F7F8F9FAFBFCFD0000"), bytes(48))
    assert ks == H("92bdd28a93c3f52511c677d08b5515a4"
                   "9da71b2378a854f67050756ded165bac"
                   "63c4868b7096d88421b563b8c94c9a31")


# test/aes.c:22-96 -- SP 800-38A F.5.1 AES-128-CTR
def test_sp800_38a_ctr():
    pt = H("6bc1bee22e409f96e93d7e117393172a"
           "ae2d8a571e03ac9c9eb76fac45af8e51"
           "30c81c46a35ce411e5fbc1191a0a52ef"
           "f69f2445df4f9b17ad2b417be66c3710")
    ct = O.aes_ctr(H("2b7e151628aed2a6abf7158809cf4f3c"),
                   H("f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff"), pt)
    assert ct == H("874d6191b620e3261bef6864990db6ce"
                   "9806f66b7970fdff8617187bb9fffdff"
                   "5ae4df3edbd5d35e5b4f09020db03eab"
                   "1e031dda2fbe03d1792170a0f3009cee")


# test/aes.c:172-396 -- AES-256-GCM vectors (the 4 success cases)
GCM_VECTORS = [
    ("b52c505a37d78eda5dd34f20c22540ea1b58963cf8e5bf8ffa85f9f2492505b4",
     "516c33929df5a3284ff463d7", "", "", "",
     "bdc1ac884d332457a1d2664f168c76f0"),
    ("31bdadd96698c204aa9ce1448ea94ae1fb4a9a0b3c9d773b51bb1822666b8f22",
     "0d18e06c7c725ac9e362e1ce", "2db5168e932556f8089a0622981d017d", "",
     "fa4362189661d163fcd6a56d8bf0405a", "d636ac1bbedd5cc3ee727dc2ab4a9489"),
    ("92e11dcdaa866f5ce790fd24501f92509aacf4cb8b1339d50c9c1240935dd08b",
     "ac93a1a6145299bde902f21a", "2d71bcfa914e4ac045b2aa60955fad24",
     "1e0889016f67601c8ebea4943bc23ad6",
     "8995ae2e6df3dbf96fac7b7137bae67f", "eca5aa77d51d4a0a14d9c51e1da474ab"),
    ("eebc1f57487f51921c0465665f8ae6d1658bb26de6f8a069a3520293a572078f",
     "99aa3e68ed8173a0eed06684", "f56e87055bc32d0eeb31b2eacc2bf2a5",
     "4d23c3cec334b49bdb370c437fec78de",
     "f7264413a84c0e7cd536867eb9f21736", "67ba0510262ae487d737ee6298f77e0c"),
]


@pytest.mark.parametrize("k,iv,pt,aad,ct,tag", GCM_VECTORS)
def test_gcm_vectors(k, iv, pt, aad, ct, tag):
    c, t = O.aes_gcm(H(k), H(iv), H(aad), H(pt))
    assert c == H(ct)
    assert t == H(tag)


# test/sha.c:17-70
SHA_DATA = [
    b"abc",
    b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
    b"9293haoijsdlasjd9ehr98wehrlsihdflskidjflaisjdlaisdjalsdkjasdlsda",
    b"9293haoijsdlasjd9ehr98wehrlsihdflskidjflaisjdlaisdjalsdkjasdlsda"
    b"9293haoijsdlasjd9ehr98wehrlsihdf",
    b"9293haoijsdlasjd9ehr98wehrlsihdflskidjflaisjdlaisdjalsdkjasdlsda"
    b"9293haoijsdlasjd82halsdlkajsdlkjasldkjasldjlskjd9ehr98wehrlsihdd",
    (b"9293haoijsdlasjd9ehr98wehrlsihdflskidjflaisjdlaisdjalsdkjasdlsda"
     b"9293haoijsdlasjd82halsdlkajsdlkjasldkjasldjlskjd9ehr98wehrlsihdd") * 2,
]
SHA_RES = [
    "a9993e364706816aba3e25717850c26c9cd0d89d",
    "84983e441c3bd26ebaae4aa1f95129e5e54670f1",
    "105104a6ee22de58c0888d2f9cdd56d95c14d4e7",
    "9962f530d85f354304efcf35ceaa29a279a3208d",
    "17307171329ed5aeaccf4cd4f6d02223a69af9fb",
    "4f051b5c4fcd0916df00f9c9dbab8608cd3355a7",
]


@pytest.mark.parametrize("i", range(len(SHA_DATA)))
def test_sha1_vectors(i):
    assert O.sha1(SHA_DATA[i]) == H(SHA_RES[i])


# test/hmac.c:22-112 -- RFC 2202 HMAC-SHA1
HMAC_VECTORS = [
    (b"\x0b" * 20, b"Hi There", "b617318655057264e28bc0b6fb378c8ef146be00"),
    (b"Jefe", b"what do ya want for nothing?",
     "effcdf6ae5eb2fa2d27416d5f184df9c259a7c79"),
    (b"\xaa" * 20, b"\xdd" * 50, "125d7342b9ac11cd91a39af48aa17b4f63f175d3"),
]


@pytest.mark.parametrize("k,d,md", HMAC_VECTORS)
def test_hmac_vectors(k, d, md):
    assert O.hmac_sha1(k, d) == H(md)


# RFC 3711 B.3 / RFC 6188 7.2 KDF vectors (test/srtp.c:197-318, #if 0'd)
def test_kdf_rfc_vectors():
    k, s = H("E1F97A0D3E018BE0D64FA32C06DE4139"), H("0EC675AD498AFEEBB6960B3AABE6")
    assert O.derive(k, s, 0, 16) == H("C61E7A93744F39EE10734AFE3FF7A087")
    assert O.derive(k, s, 1, 20) == H("CEBE321F6FF7716B6FD4AB49AF256A156D38BAA4")
    assert O.derive(k, s, 2, 14) == H("30CBBC08863D8C85D49DB34A9AE1")
    assert O.derive(k, s, 3, 16) == H("4c1aa45a81f73d61c800bbb00fbb1eaa")
    assert O.derive(k, s, 4, 20) == H("8d54534feb49ae8e7993a6bd0b844fc323a93dfd")
    assert O.derive(k, s, 5, 14) == H("9581c7ad87b3e530bf3e4454a8b3")
    k = H("f0f04914b513f2763a1b1fa130f10e2998f6f6e43e4309d1e622a0e332b9f1b6")
    s = H("3b04803de51ee7c96423ab5b78d2")
    assert O.derive(k, s, 0, 32) == H("5ba1064e30ec51613cad926c5a28ef73"
                                      "1ec7fb397f70a960653caf06554cd8c4")
    assert O.derive(k, s, 1, 20) == H("fd9c32d39ed5fbb5a9dc96b30818454d1313dc05")
    assert O.derive(k, s, 2, 14) == H("fa31791685ca444a9e07c6c64e93")


def test_golden_primitives(golden):
    for v in golden["kdf"]:
        assert O.derive(H(v["key"]), H(v["salt"]), v["label"],
                        len(v["out"]) // 2) == H(v["out"])
    for v in golden["gcm"]:
        c, t = O.aes_gcm(H(v["key"]), H(v["iv"]), H(v["aad"]), H(v["pt"]))
        assert c == H(v["ct"]) and t == H(v["tag"])
    for v in golden["hmac"]:
        if v["data"]:
            assert O.hmac_sha1(H(v["key"]), H(v["data"])) == H(v["mac"])


def test_alloc_errors_and_names(golden):
    import ctypes
    be = O.OracleBackend()
    for suite, klen, err in golden["alloc"]:
        p = ctypes.c_void_p()
        e = be.l.oracle_srtp_alloc(ctypes.byref(p), suite, bytes(64), klen, 0)
        assert e == err, (suite, klen)
        if not e:
            be.free(p)
    names = [be.l.oracle_srtp_suite_name(s).decode() for s in range(-1, 8)]
    assert names == golden["names"]


# test/srtp.c:514-570 / 583-632 -- libsrtp full-packet known answers
def test_libsrtp_packets():
    be = O.OracleBackend()
    key = b"\x22" * 16 + b"\x44" * 14
    ctx, err = be.alloc(1, key, 0)
    assert err == 0
    pkt = H("800000010000000001020304") + b"\xa5" * 20
    e, pos, end, size, buf = be.call(ctx, "srtp_encrypt", 512, 0, 32, pkt, 0)
    assert e == 0 and buf[:end] == H(
        "800000010000000001020304f5b44b7e3ad4eb057bc6480c45df6547bb70bcc2"
        "7b136e1f3d3a62821b15")
    be.free(ctx)
    ctx, err = be.alloc(0, key, 0)
    e, pos, end, size, buf = be.call(ctx, "srtcp_encrypt", 512, 0, 12,
                                     H("81cb00020102030401620000"), 0)
    assert e == 0 and buf[:end] == H("81cb00020102030487c9fcdb80000001e9442fcc")
    be.free(ctx)


def test_golden_scenarios(golden):
    be = O.OracleBackend()
    bad = [m for m in (replay_scenario(be, s) for s in golden["scenarios"])
           if m]
    assert not bad, bad[:5]
