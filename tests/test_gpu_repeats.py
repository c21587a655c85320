"""k_long's pass-2 CheapRepWordsInplace (compact_lang_det_impl.cc:610-692) runs
over the span cache with the predictor in LDS as 16-bit codes (lng::pred_code):
one-to-one on 1-byte, 2-byte and well-formed 3-byte characters, a sentinel
class (4-byte and malformed characters) whose full value lives in the slot.
These documents put every class into the predictor, with repeated words so
that entries are both hit and rewritten, and check the HIP path against the
oracle bit for bit (needs an MI355X)."""
import numpy as np
import pytest

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

# words per class: ASCII, 2-byte (Cyrillic, Latin-1), 3-byte (Devanagari, Han,
# the top of the BMP), 4-byte (Han extension B, Gothic), mixed
WORDS = {
    "latin": ["the", "quick", "brown", "fox", "jumps", "over", "lazy", "dog", "and", "runs"],
    "accent": ["été", "déjà", "naïve", "façade", "über", "größe", "señor", "año", "mañana", "crème"],
    "cyr": ["привет", "мир", "дом", "кот", "собака", "улица", "город", "вода", "хлеб", "снег"],
    "deva": ["नमस्ते", "दुनिया", "घर", "पानी", "किताब", "भारत", "समय", "लोग", "काम", "दिन"],
    "han": ["我们", "你好", "世界", "中国", "学习", "语言", "时间", "朋友", "工作", "问题"],
    "extb": ["\U00020000\U00020001", "\U00020002我", "\U0002A6D6\U00020003", "你\U00020004",
             "\U00020005\U00020006\U00020007", "\U00024000", "\U00020010好", "\U00020020\U00020021"],
    "gothic": ["\U00010330\U00010331\U00010332", "\U00010333\U00010334", "\U00010335\U00010336\U00010337\U00010338"],
    "bmp_top": ["￠ａ", "ｂｃ", "ﬁﬂ"],
}


def make_doc(rng, kinds, n_words, repeat):
    """Paragraphs of each kind; `repeat` = chance a word repeats a recent one
    (drives predictions and deletions)."""
    parts = []
    for kind in kinds:
        vocab = WORDS[kind]
        out = []
        for _ in range(n_words):
            if out and rng.random() < repeat:
                out.append(out[-int(rng.integers(1, min(len(out), 4) + 1))])
            else:
                out.append(vocab[int(rng.integers(len(vocab)))])
        parts.append(" ".join(out))
    return ("\n".join(parts) + "\n").encode("utf-8")


def test_repeats_predictor_code_classes(gpu, oracle):
    rng = np.random.default_rng(23)
    mixes = [["latin", "accent"], ["cyr", "latin"], ["deva", "cyr"], ["han", "extb"], ["extb", "han", "latin"],
             ["gothic", "latin"], ["bmp_top", "han"], ["accent", "cyr", "deva", "han", "extb", "gothic"]]
    docs = []
    for i in range(600):
        kinds = mixes[i % len(mixes)]
        docs.append(make_doc(rng, kinds, int(rng.integers(40, 400)), float(rng.choice([0.0, 0.3, 0.7, 0.95]))))
    # malformed sequences inside letter runs (stray continuation bytes, cut and
    # overlong forms), kept away from the document end
    for i in range(0, len(docs), 5):
        d = bytearray(docs[i])
        for _ in range(3):
            p = int(rng.integers(1, max(2, len(d) - 8)))
            d[p:p] = rng.choice([b"\x80", b"\xc3", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf0\x9f"])
        docs[i] = bytes(d)
    buf, offs = gpu.pack(docs)
    got = gpu.detect_batch(buf=buf, offsets=offs)
    st = gpu.last_stats(0)
    assert st.long_docs > 300                 # the long-document kernel took most of them
    assert st.passes[1] > 100                 # and many went through the Repeats pass
    assert_same(got, oracle.detect_batch(buf, offs, threads=8), "repeats code classes")
