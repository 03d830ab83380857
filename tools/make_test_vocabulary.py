"""Build the small test vocabulary tests/golden/test_voc_k10l6.txt (DBoW2 text format).

The reference runs with whatever ORB vocabulary System is given (System.cc:67,
TemplatedVocabulary::loadFromTextFile, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424);
its ORBvoc.txt is missing from the checkout (.MISSING_LARGE_BLOBS).  This script trains a small
vocabulary in the same file format -- header "k L scoring weighting", then one line per node in
id order: "parent is_leaf d0 .. d31 weight" -- by hierarchical k-medians over ORB descriptors,
the way DBoW2's create() does (HKmeansStep: k-means++ seeding, Hamming assignment, bitwise
majority means, children of a node contiguous and created depth-first; a cluster of at most k
descriptors becomes k leaves), with TF-IDF word weights log(N / n_i) over the N training images.

Training data: the ORB descriptors (oracle extractor, 2000 features) of kitti_sample frames 0, 2,
4 and of three frames of the synthetic street scene with seeds that no test or bench sequence
uses.  k = 10 and L = 6 as ORBvoc.txt, so transform(..., levelsup = 4) files features under
level-2 nodes, as the reference's 4-levels-up FeatureVector does.  The tree is ragged: a cluster of more than 20
descriptors is split again down to level 4, so the words (leaves at levels 3 and 4, about 12
descriptors each) recur across the training images and their IDF weights differ (a word seen in
every image weighs 0 and is stopped, as DBoW2 does).  The file is written without a trailing newline: loadFromTextFile's
`while(!f.eof())` reads one extra empty line otherwise and links an uninitialised parent.

  python tools/make_test_vocabulary.py            # writes tests/golden/test_voc_k10l6.txt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

OUT = os.path.join(ROOT, "tests", "golden", "test_voc_k10l6.txt")
K, L = 10, 6
MAX_DEPTH, MIN_SPLIT = 4, 20  # leaves at level 3 or 4: words shared between images


def hamming(bits, centres):
    """bits (n, 256) bool, centres (k, 256) bool -> (n, k) distances."""
    return (bits[:, None, :] != centres[None, :, :]).sum(-1)


def kmeans(bits, k, rng, iters=8):
    n = len(bits)
    # k-means++ seeding (DBoW2 initiateClustersKMpp)
    c = [int(rng.integers(n))]
    d = hamming(bits, bits[c]).min(1).astype(np.float64)
    while len(c) < k:
        if d.sum() == 0:
            break
        p = d ** 2 / (d ** 2).sum()
        c.append(int(rng.choice(n, p=p)))
        d = np.minimum(d, hamming(bits, bits[c[-1:]])[:, 0])
    centres = bits[c].copy()
    assign = None
    for _ in range(iters):
        a = hamming(bits, centres).argmin(1)
        if assign is not None and np.array_equal(a, assign):
            break
        assign = a
        for j in range(len(centres)):
            m = bits[a == j]
            if len(m):  # FORB::meanValue: bit set where at least half the descriptors have it
                centres[j] = m.sum(0) >= (len(m) + 1) // 2
    a = hamming(bits, centres).argmin(1)
    return centres, a


def build(desc, img_of, n_images, seed=7):
    rng = np.random.default_rng(seed)
    bits = np.unpackbits(desc, axis=1, bitorder="big").astype(bool)
    nodes = [None]  # node 0: root; entries (parent, bits, members)
    children = {0: []}

    def step(parent, idx, level):
        if len(idx) <= K:
            cent = [bits[i] for i in idx]
            groups = [[i] for i in idx]
        else:
            centres, a = kmeans(bits[idx], K, rng)
            cent, groups = [], []
            for j in range(len(centres)):
                g = idx[a == j]
                if len(g):
                    cent.append(centres[j])
                    groups.append(g)
        ids = []
        for cb, g in zip(cent, groups):
            nodes.append((parent, cb, np.asarray(g)))
            nid = len(nodes) - 1
            children[nid] = []
            children[parent].append(nid)
            ids.append(nid)
        if level < min(L, MAX_DEPTH):
            for nid, g in zip(ids, groups):
                if len(g) > MIN_SPLIT:
                    step(nid, np.asarray(g), level + 1)

    step(0, np.arange(len(desc)), 1)
    lines = []
    for nid in range(1, len(nodes)):
        parent, cb, members = nodes[nid]
        leaf = len(children[nid]) == 0
        w = 0.0
        if leaf:
            ni = len(np.unique(img_of[members]))
            w = float(np.log(n_images / ni))
        d = np.packbits(cb.astype(np.uint8), bitorder="big")
        lines.append("%d %d %s %.17g" % (parent, 1 if leaf else 0,
                                         " ".join(str(int(v)) for v in d), w))
    return "%d %d  %d %d\n" % (K, L, 0, 0) + "\n".join(lines)


def training_descriptors():
    import torch
    from conftest import load_kitti_frame
    from multimot_track_amd import scene
    from oracle import oracle as O
    O.build()
    descs, imgs = [], []
    grays = [O.gray_from_bgr(load_kitti_frame(i)["bgr"]) for i in (0, 2, 4)]
    for s in (71, 72, 73):
        seq = scene.kitti_like_sequence(1, 1242, 375, n_objects=3, seed=s, device="cpu", start=40)
        grays.append(O.gray_from_bgr(seq["bgr"][0].numpy()))
    for g in grays:
        _, d = O.orb_extract(g, 2000)
        descs.append(d)
        imgs.append(np.full(len(d), len(imgs)))
    torch.set_num_threads(1)
    return np.concatenate(descs), np.concatenate(imgs), len(grays)


def main():
    desc, img_of, n = training_descriptors()
    text = build(desc, img_of, n)
    with open(OUT, "w") as f:
        f.write(text)
    print("%s: %d nodes from %d descriptors of %d images" % (OUT, text.count("\n"), len(desc), n))


if __name__ == "__main__":
    main()
