"""paddle.text: viterbi decoding + dataset readers. Reference: python/paddle/text/ (viterbi_decode.py
ViterbiDecoder / viterbi_decode; datasets/: Imdb, Imikolov, Movielens, UCIHousing, WMT14, WMT16, Conll05).
Datasets read local copies only (no network)."""
from __future__ import annotations

import os
import tarfile

import numpy as np
import torch

from .. import nn
from ..framework.tensor import Tensor, _wrap
from ..io import Dataset


def viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag=True, name=None):
    """potentials [B, T, N], transitions [N, N], lengths [B] -> (scores [B], paths [B, T])."""
    emit = potentials._t.float()
    trans = transition_params._t.float()
    lens = lengths._t.long()
    B, T, N = emit.shape
    if include_bos_eos_tag:
        # tags N-2 = BOS, N-1 = EOS (reference convention)
        start = trans[N - 2].clone()
        stop = trans[:, N - 1].clone()
    else:
        start = torch.zeros(N, device=emit.device)
        stop = torch.zeros(N, device=emit.device)
    alpha = emit[:, 0] + start
    back = []
    for t in range(1, T):
        score = alpha[:, :, None] + trans[None]  # [B, from, to]
        best, arg = score.max(1)
        new = best + emit[:, t]
        active = (t < lens)[:, None]
        alpha = torch.where(active, new, alpha)
        back.append(torch.where(active, arg, torch.arange(N, device=emit.device).expand(B, N)))
    alpha = alpha + stop
    scores, last = alpha.max(-1)
    path = [last]
    for bp in reversed(back):
        last = bp.gather(1, last[:, None])[:, 0]
        path.append(last)
    path = torch.stack(path[::-1], 1)
    # positions beyond each length are padding: zero them
    mask = torch.arange(T, device=emit.device)[None] < lens[:, None]
    return _wrap(scores), _wrap(torch.where(mask, path, torch.zeros_like(path)))


class ViterbiDecoder(nn.Layer):
    def __init__(self, transitions, include_bos_eos_tag=True, name=None):
        super().__init__()
        self.transitions = transitions
        self.include_bos_eos_tag = include_bos_eos_tag

    def forward(self, potentials, lengths):
        return viterbi_decode(potentials, self.transitions, lengths, self.include_bos_eos_tag)


def _need(p, what):
    if p is None or not os.path.exists(p):
        raise FileNotFoundError(f"{what}: local file {p!r} not found (no network; downloads are disabled)")


class UCIHousing(Dataset):
    """whitespace-separated 14-column housing data file."""

    def __init__(self, data_file=None, mode="train", download=False):
        _need(data_file, "UCIHousing")
        data = np.loadtxt(data_file).astype("float32").reshape(-1, 14)
        mx, mn, avg = data.max(0), data.min(0), data.mean(0)
        feats = (data[:, :13] - avg[:13]) / (mx[:13] - mn[:13])
        data = np.concatenate([feats, data[:, 13:]], 1)
        cut = int(len(data) * 0.8)
        self.data = data[:cut] if mode == "train" else data[cut:]

    def __getitem__(self, idx):
        d = self.data[idx]
        return d[:-1], d[-1:]

    def __len__(self):
        return len(self.data)


class Imdb(Dataset):
    """aclImdb tarball: reviews tokenised on whitespace/punctuation, word dict built from train."""

    def __init__(self, data_file=None, mode="train", cutoff=150, download=False):
        _need(data_file, "Imdb")
        import re
        self.docs, self.labels = [], []
        pat = re.compile(rf"aclImdb/{mode}/(pos|neg)/.*\.txt$")
        freq = {}
        raw = []
        with tarfile.open(data_file) as tf:
            for m in tf.getmembers():
                g = pat.match(m.name)
                if g:
                    words = re.sub(r"[^\w\s]", " ", tf.extractfile(m).read().decode("utf-8", "ignore").lower()).split()
                    raw.append((words, 0 if g.group(1) == "pos" else 1))
                    for w in words:
                        freq[w] = freq.get(w, 0) + 1
        vocab = sorted([w for w, c in freq.items() if c > cutoff], key=lambda w: (-freq[w], w))
        self.word_idx = {w: i for i, w in enumerate(vocab)}
        unk = len(self.word_idx)
        self.word_idx["<unk>"] = unk
        for words, lab in raw:
            self.docs.append(np.array([self.word_idx.get(w, unk) for w in words], dtype="int64"))
            self.labels.append(np.array([lab], dtype="int64"))

    def __getitem__(self, idx):
        return self.docs[idx], self.labels[idx]

    def __len__(self):
        return len(self.docs)


class Imikolov(Dataset):
    def __init__(self, data_file=None, data_type="NGRAM", window_size=-1, mode="train", min_word_freq=50,
                 download=False):
        _need(data_file, "Imikolov")
        name = {"train": "ptb.train.txt", "test": "ptb.valid.txt"}[mode]
        with tarfile.open(data_file) as tf:
            text = [m for m in tf.getmembers() if m.name.endswith(name)]
            lines = tf.extractfile(text[0]).read().decode().splitlines()
        freq = {}
        for l in lines:
            for w in l.split():
                freq[w] = freq.get(w, 0) + 1
        vocab = sorted([w for w, c in freq.items() if c >= min_word_freq], key=lambda w: (-freq[w], w))
        self.word_idx = {w: i for i, w in enumerate(vocab)}
        for s in ("<s>", "<e>", "<unk>"):
            self.word_idx.setdefault(s, len(self.word_idx))
        unk = self.word_idx["<unk>"]
        self.data = []
        for l in lines:
            ids = [self.word_idx["<s>"]] + [self.word_idx.get(w, unk) for w in l.split()] + [self.word_idx["<e>"]]
            if data_type == "NGRAM":
                for i in range(window_size, len(ids) + 1):
                    self.data.append(tuple(np.array([x]) for x in ids[i - window_size:i]))
            else:
                self.data.append((np.array(ids[:-1]), np.array(ids[1:])))

    def __getitem__(self, idx):
        return self.data[idx]

    def __len__(self):
        return len(self.data)


# ---------------------------------------------------------------------------------------------- Movielens
_AGES = (1, 18, 25, 35, 45, 50, 56)


class Movielens(Dataset):
    """MovieLens-1M ratings from the local ``ml-1m.zip`` (``ml-1m/{movies,users,ratings}.dat``, '::'-separated,
    latin-1). Sample = (user id, gender 0 = M / 1 = F, age bucket, job, movie id, category ids, title word ids,
    rating * 2 - 5). Ratings go to train / test by a seeded uniform draw per line (``test_ratio``).
    Category and title-word ids are assigned in sorted order (deterministic across processes).
    Reference: python/paddle/text/datasets/movielens.py."""

    def __init__(self, data_file=None, mode="train", test_ratio=0.1, rand_seed=0, download=False):
        import re
        import zipfile
        if mode.lower() not in ("train", "test"):
            raise ValueError(f"mode should be 'train' or 'test', got {mode}")
        _need(data_file, "Movielens")
        self.data_file, self.mode = data_file, mode.lower()
        title_re = re.compile(r"^(.*)\((\d+)\)$")
        with zipfile.ZipFile(data_file) as z:
            movies, cats, words = {}, set(), set()
            for line in z.read("ml-1m/movies.dat").decode("latin-1").splitlines():
                if not line.strip():
                    continue
                mid, title, cat = line.strip().split("::")
                m = title_re.match(title)
                title = m.group(1) if m else title
                cs = cat.split("|")
                movies[int(mid)] = (cs, title)
                cats.update(cs)
                words.update(w.lower() for w in title.split())
            self.categories_dict = {c: i for i, c in enumerate(sorted(cats))}
            self.movie_title_dict = {w: i for i, w in enumerate(sorted(words))}
            self.movie_info = {k: ([k], [self.categories_dict[c] for c in cs],
                                   [self.movie_title_dict[w.lower()] for w in t.split()])
                               for k, (cs, t) in movies.items()}
            self.user_info = {}
            for line in z.read("ml-1m/users.dat").decode("latin-1").splitlines():
                if not line.strip():
                    continue
                uid, gender, age, job = line.strip().split("::")[:4]
                self.user_info[int(uid)] = [[int(uid)], [0 if gender == "M" else 1], [_AGES.index(int(age))],
                                            [int(job)]]
            rng = np.random.RandomState(rand_seed)
            is_test = self.mode == "test"
            self.data = []
            for line in z.read("ml-1m/ratings.dat").decode("latin-1").splitlines():
                if not line.strip():
                    continue
                if (rng.random_sample() < test_ratio) != is_test:
                    continue
                uid, mid, rating = line.strip().split("::")[:3]
                self.data.append(self.user_info[int(uid)] + list(self.movie_info[int(mid)])
                                 + [[float(rating) * 2 - 5.0]])

    def __getitem__(self, idx):
        return tuple(np.array(d) for d in self.data[idx])

    def __len__(self):
        return len(self.data)


# ---------------------------------------------------------------------------------------------- WMT14 / WMT16
def _seq_triplet(src_words, trg_words, src_dict, trg_dict, start, end, unk):
    src = [src_dict.get(w, unk) for w in [start] + src_words + [end]]
    trg = [trg_dict.get(w, unk) for w in trg_words]
    return src, [trg_dict[start]] + trg, trg + [trg_dict[end]]


class _ParallelText(Dataset):
    def __getitem__(self, idx):
        return np.array(self.src_ids[idx]), np.array(self.trg_ids[idx]), np.array(self.trg_ids_next[idx])

    def __len__(self):
        return len(self.src_ids)


class WMT14(_ParallelText):
    """WMT14 en-fr from the local tarball: ``*src.dict`` / ``*trg.dict`` (one word per line, the first
    ``dict_size`` kept), ``<mode>/<mode>`` files of 'src\\ttrg' lines. Pairs with a side longer than 80 ids are
    dropped. <s> / <e> wrap the source; the target comes as (<s> + trg, trg + <e>); unknown words -> id 2.
    Reference: python/paddle/text/datasets/wmt14.py."""

    def __init__(self, data_file=None, mode="train", dict_size=-1, download=False):
        if mode.lower() not in ("train", "test", "gen"):
            raise ValueError(f"mode should be 'train', 'test' or 'gen', got {mode}")
        if dict_size <= 0:
            raise ValueError("dict_size should be set as positive number")
        _need(data_file, "WMT14")
        self.mode, self.dict_size, self.data_file = mode.lower(), dict_size, data_file
        self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
        with tarfile.open(data_file) as tf:
            members = tf.getmembers()

            def read_dict(suffix):
                m = [x for x in members if x.name.endswith(suffix)]
                if len(m) != 1:
                    raise ValueError(f"WMT14: expected one *{suffix} in the archive, found {len(m)}")
                out = {}
                for i, line in enumerate(tf.extractfile(m[0])):
                    if i >= dict_size:
                        break
                    out[line.strip().decode()] = i
                return out
            self.src_dict, self.trg_dict = read_dict("src.dict"), read_dict("trg.dict")
            for m in members:
                if not m.name.endswith(f"{self.mode}/{self.mode}"):
                    continue
                for line in tf.extractfile(m):
                    parts = line.decode().strip().split("\t")
                    if len(parts) != 2:
                        continue
                    s, t, tn = _seq_triplet(parts[0].split(), parts[1].split(), self.src_dict, self.trg_dict,
                                            "<s>", "<e>", 2)
                    if len(s) > 80 or len(t) - 1 > 80:
                        continue
                    self.src_ids.append(s)
                    self.trg_ids.append(t)
                    self.trg_ids_next.append(tn)


class WMT16(_ParallelText):
    """WMT16 en-de (Multi30k) from the local tarball: ``wmt16/{train,val,test}`` files of 'en\\tde' lines.
    Each language's dictionary is <s>, <e>, <unk>, then the most frequent words of that language's column of
    ``wmt16/train`` (ties by first appearance), ``dict_size`` entries in all; built in memory (and cached
    next to the archive as ``<lang>_<size>.dict`` when the directory is writable).
    Reference: python/paddle/text/datasets/wmt16.py."""

    TOTAL = {"en": 11250, "de": 19220}

    def __init__(self, data_file=None, mode="train", src_dict_size=-1, trg_dict_size=-1, lang="en", download=False):
        if mode.lower() not in ("train", "test", "val"):
            raise ValueError(f"mode should be 'train', 'test' or 'val', got {mode}")
        if src_dict_size <= 0 or trg_dict_size <= 0:
            raise ValueError("dict_size should be set as positive number")
        if lang not in ("en", "de"):
            raise ValueError("lang should be 'en' or 'de'")
        _need(data_file, "WMT16")
        self.mode, self.lang, self.data_file = mode.lower(), lang, data_file
        other = "de" if lang == "en" else "en"
        self.src_dict_size = min(src_dict_size, self.TOTAL[lang])
        self.trg_dict_size = min(trg_dict_size, self.TOTAL[other])
        with tarfile.open(data_file) as tf:
            train = [l.decode().strip().split("\t") for l in tf.extractfile("wmt16/train")]
            rows = [l.decode().strip().split("\t") for l in tf.extractfile(f"wmt16/{self.mode}")]
        train = [p for p in train if len(p) == 2]
        self.src_dict = self._build_dict(train, lang, self.src_dict_size)
        self.trg_dict = self._build_dict(train, other, self.trg_dict_size)
        sc = 0 if lang == "en" else 1
        self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
        for p in rows:
            if len(p) != 2:
                continue
            s, t, tn = _seq_triplet(p[sc].split(), p[1 - sc].split(), self.src_dict, self.trg_dict, "<s>", "<e>",
                                    self.src_dict["<unk>"])
            self.src_ids.append(s)
            self.trg_ids.append(t)
            self.trg_ids_next.append(tn)

    def _build_dict(self, train, lang, size):
        col = 0 if lang == "en" else 1
        counts = {}
        for p in train:
            for w in p[col].split():
                counts[w] = counts.get(w, 0) + 1
        words = ["<s>", "<e>", "<unk>"] + [w for w, _ in sorted(counts.items(), key=lambda kv: -kv[1])]
        words = words[:size]
        path = os.path.join(os.path.dirname(os.path.abspath(self.data_file)), f"{lang}_{size}.dict")
        try:
            with open(path, "w") as f:
                f.write("\n".join(words) + "\n")
        except OSError:
            pass
        return {w: i for i, w in enumerate(words)}

    def get_dict(self, lang, reverse=False):
        d = self.src_dict if lang == self.lang else self.trg_dict
        return {i: w for w, i in d.items()} if reverse else dict(d)


# ---------------------------------------------------------------------------------------------- Conll05
class Conll05st(Dataset):
    """CoNLL-2005 SRL test.wsj from the local ``conll05st-tests.tar.gz`` (gzipped words / props files) plus
    the word / verb / target dictionaries. One sample per predicate of a sentence: (word ids, the 5 context
    word ids around the predicate broadcast over the sentence, predicate id, context mark, BIO label ids).
    Unknown words -> 0. Reference: python/paddle/text/datasets/conll05.py."""

    WORDS = "conll05st-release/test.wsj/words/test.wsj.words.gz"
    PROPS = "conll05st-release/test.wsj/props/test.wsj.props.gz"

    def __init__(self, data_file=None, word_dict_file=None, verb_dict_file=None, target_dict_file=None,
                 emb_file=None, download=False):
        import gzip
        for p, n in ((data_file, "data_file"), (word_dict_file, "word_dict_file"), (verb_dict_file, "verb_dict_file"),
                     (target_dict_file, "target_dict_file")):
            _need(p, f"Conll05st {n}")
        self.data_file, self.emb_file = data_file, emb_file
        self.word_dict = self._load_dict(word_dict_file)
        self.predicate_dict = self._load_dict(verb_dict_file)
        tags = []
        with open(target_dict_file) as f:
            for line in f:
                line = line.strip()
                if line[:2] in ("B-", "I-") and line[2:] not in tags:
                    tags.append(line[2:])
        self.label_dict = {}
        for t in tags:
            self.label_dict["B-" + t] = len(self.label_dict)
            self.label_dict["I-" + t] = len(self.label_dict)
        self.label_dict["O"] = len(self.label_dict)
        self.sentences, self.predicates, self.labels = [], [], []
        with tarfile.open(data_file) as tf:
            words = gzip.decompress(tf.extractfile(self.WORDS).read()).decode().splitlines()
            props = gzip.decompress(tf.extractfile(self.PROPS).read()).decode().splitlines()
        sent, cols = [], []
        for w, pr in zip(words, props):
            fields = pr.split()
            if not fields:
                self._add_sentence(sent, cols)
                sent, cols = [], []
            else:
                sent.append(w.strip())
                cols.append(fields)
        if sent:
            self._add_sentence(sent, cols)

    @staticmethod
    def _load_dict(path):
        with open(path) as f:
            return {line.strip(): i for i, line in enumerate(f)}

    def _add_sentence(self, sent, cols):
        if not cols:
            return
        columns = list(zip(*cols))
        verbs = [x for x in columns[0] if x != "-"]
        for k, col in enumerate(columns[1:]):
            seq, tag, open_ = [], "O", False
            for tok in col:
                if tok == "*":
                    seq.append("I-" + tag if open_ else "O")
                elif tok == "*)":
                    seq.append("I-" + tag)
                    open_ = False
                elif "(" in tok:
                    tag = tok[1:tok.index("*")]
                    seq.append("B-" + tag)
                    open_ = ")" not in tok
                else:
                    raise RuntimeError(f"Conll05st: unexpected label {tok!r}")
            self.sentences.append(sent)
            self.predicates.append(verbs[k])
            self.labels.append(seq)

    def __getitem__(self, idx):
        sent, pred, labels = self.sentences[idx], self.predicates[idx], self.labels[idx]
        n = len(sent)
        v = labels.index("B-V")
        mark = [0] * n
        ctx = {}
        for off, name, pad in ((-2, "n2", "bos"), (-1, "n1", "bos"), (0, "0", None), (1, "p1", "eos"),
                               (2, "p2", "eos")):
            j = v + off
            if 0 <= j < n:
                mark[j] = 1
                ctx[name] = sent[j]
            else:
                ctx[name] = pad
        wd = self.word_dict
        rep = lambda w: np.array([wd.get(w, 0)] * n)  # noqa: E731
        return (np.array([wd.get(w, 0) for w in sent]), rep(ctx["n2"]), rep(ctx["n1"]), rep(ctx["0"]),
                rep(ctx["p1"]), rep(ctx["p2"]), np.array([self.predicate_dict.get(pred)] * n), np.array(mark),
                np.array([self.label_dict.get(l) for l in labels]))

    def __len__(self):
        return len(self.sentences)

    def get_dict(self):
        return self.word_dict, self.predicate_dict, self.label_dict

    def get_embedding(self):
        return self.emb_file


class datasets:  # paddle.text.datasets namespace
    UCIHousing = UCIHousing
    Imdb = Imdb
    Imikolov = Imikolov
    Movielens = Movielens
    WMT14 = WMT14
    WMT16 = WMT16
    Conll05st = Conll05st
