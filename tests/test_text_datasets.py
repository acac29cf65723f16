"""Text dataset readers on small synthetic archives in the reference's layouts (the real archives are
downloads; there is no network): Movielens (ml-1m zip), WMT14 / WMT16 (tarballs), Conll05st (tar.gz of gzipped
words / props + dictionaries). Parity unpinned against the reference's own outputs (they need the real data)."""
import gzip
import io
import tarfile
import zipfile

import numpy as np
import pytest

import paddlepaddle_amd as paddle


def _tar_add(tf, name, data):
    info = tarfile.TarInfo(name)
    info.size = len(data)
    tf.addfile(info, io.BytesIO(data))


def test_movielens(tmp_path):
    p = tmp_path / "ml-1m.zip"
    with zipfile.ZipFile(p, "w") as z:
        z.writestr("ml-1m/movies.dat", "1::Toy Story (1995)::Animation|Comedy\n2::Heat (1995)::Action\n")
        z.writestr("ml-1m/users.dat", "1::F::1::10::48067\n2::M::56::16::70072\n")
        z.writestr("ml-1m/ratings.dat", "".join(f"{1 + i % 2}::{1 + (i // 2) % 2}::{1 + i % 5}::97830{i}\n"
                                                for i in range(40)))
    tr = paddle.text.datasets.Movielens(data_file=str(p), mode="train", test_ratio=0.25)
    te = paddle.text.datasets.Movielens(data_file=str(p), mode="test", test_ratio=0.25)
    assert len(tr) + len(te) == 40 and len(te) > 0
    uid, gender, age, job, mid, cats, title, rating = tr[0]
    assert uid.tolist() == [1] and gender.tolist() == [1] and age.tolist() == [0] and job.tolist() == [10]
    assert mid.tolist() == [1]
    assert cats.tolist() == [tr.categories_dict["Animation"], tr.categories_dict["Comedy"]]
    assert title.tolist() == [tr.movie_title_dict["toy"], tr.movie_title_dict["story"]]
    assert rating.tolist() == [1.0 * 2 - 5.0]


def _wmt14(tmp_path):
    p = tmp_path / "wmt14.tgz"
    src = "<s>\n<e>\n<unk>\nle\nchat\nnoir\n"
    trg = "<s>\n<e>\n<unk>\nthe\ncat\nblack\n"
    with tarfile.open(p, "w:gz") as tf:
        _tar_add(tf, "wmt14/src.dict", src.encode())
        _tar_add(tf, "wmt14/trg.dict", trg.encode())
        _tar_add(tf, "wmt14/train/train", b"le chat noir\tthe black cat\nle chien\tthe dog\nbad line\n")
        _tar_add(tf, "wmt14/test/test", b"le chat\tthe cat\n")
    return p


def test_wmt14(tmp_path):
    ds = paddle.text.datasets.WMT14(data_file=str(_wmt14(tmp_path)), mode="train", dict_size=6)
    assert len(ds) == 2
    s, t, tn = ds[0]
    assert s.tolist() == [0, 3, 4, 5, 1] and t.tolist() == [0, 3, 5, 4] and tn.tolist() == [3, 5, 4, 1]
    s, t, tn = ds[1]
    assert s.tolist() == [0, 3, 2, 1] and t.tolist() == [0, 3, 2]   # unknown words -> 2
    small = paddle.text.datasets.WMT14(data_file=str(_wmt14(tmp_path)), mode="test", dict_size=4)
    assert small[0][0].tolist() == [0, 3, 2, 1]
    with pytest.raises(ValueError):
        paddle.text.datasets.WMT14(data_file=str(_wmt14(tmp_path)), dict_size=-1)


def test_wmt16(tmp_path):
    p = tmp_path / "wmt16.tar.gz"
    train = "a cat sat\teine katze sass\na dog sat\tein hund sass\na cat ran\teine katze lief\n"
    with tarfile.open(p, "w:gz") as tf:
        _tar_add(tf, "wmt16/train", train.encode())
        _tar_add(tf, "wmt16/val", b"a cat\teine katze\n")
        _tar_add(tf, "wmt16/test", b"the bird\tder vogel\n")
    ds = paddle.text.datasets.WMT16(data_file=str(p), mode="val", src_dict_size=6, trg_dict_size=5, lang="en")
    en, de = ds.get_dict("en"), ds.get_dict("de")
    assert list(en)[:3] == ["<s>", "<e>", "<unk>"] and en["a"] == 3 and len(en) == 6
    assert de["eine"] == 3 or de["katze"] == 3  # most frequent German words first
    s, t, tn = ds[0]
    assert s.tolist() == [0, en["a"], en["cat"], 1] and t.tolist() == [0, de["eine"], de["katze"]]
    assert tn.tolist() == [de["eine"], de["katze"], 1]
    rev = paddle.text.datasets.WMT16(data_file=str(p), mode="test", src_dict_size=6, trg_dict_size=5, lang="de")
    assert rev[0][0].tolist() == [0, 2, 2, 1]   # unknown German words on the source side


def test_conll05(tmp_path):
    words = "The\ncat\nsat\n.\n\n"
    # two predicates in one sentence: columns 2 and 3
    props = "-\t(A0*\t*\n-\t*)\t(V*)\nsit\t(V*)\t(A1*\nrun\t*\t*)\n\n"
    data = tmp_path / "conll05st-tests.tar.gz"
    with tarfile.open(data, "w:gz") as tf:
        _tar_add(tf, "conll05st-release/test.wsj/words/test.wsj.words.gz", gzip.compress(words.encode()))
        _tar_add(tf, "conll05st-release/test.wsj/props/test.wsj.props.gz", gzip.compress(props.encode()))
    wd = tmp_path / "wordDict.txt"
    wd.write_text("<unk>\nThe\ncat\nsat\n.\nbos\neos\n")
    vd = tmp_path / "verbDict.txt"
    vd.write_text("sit\nrun\n")
    td = tmp_path / "targetDict.txt"
    td.write_text("B-A0\nI-A0\nB-A1\nI-A1\nB-V\nI-V\nO\n")
    ds = paddle.text.datasets.Conll05st(data_file=str(data), word_dict_file=str(wd), verb_dict_file=str(vd),
                                        target_dict_file=str(td))
    assert len(ds) == 2
    w, n2, n1, c0, p1, p2, pred, mark, lab = ds[0]
    _, _, ld = ds.get_dict()
    assert w.tolist() == [1, 2, 3, 4]
    assert c0.tolist() == [3] * 4 and n1.tolist() == [2] * 4 and n2.tolist() == [1] * 4
    assert p1.tolist() == [4] * 4 and p2.tolist() == [6] * 4   # past the end -> "eos"
    assert pred.tolist() == [0] * 4 and mark.tolist() == [1, 1, 1, 1]
    assert lab.tolist() == [ld["B-A0"], ld["I-A0"], ld["B-V"], ld["O"]]
    w, n2, n1, c0, p1, p2, pred, mark, lab = ds[1]
    assert pred.tolist() == [1] * 4 and c0.tolist() == [2] * 4 and n2.tolist() == [5] * 4   # "bos"
    assert lab.tolist() == [ld["O"], ld["B-V"], ld["B-A1"], ld["I-A1"]]


def test_missing_archive_is_a_clear_error():
    with pytest.raises(FileNotFoundError):
        paddle.text.datasets.Movielens(data_file=None)
