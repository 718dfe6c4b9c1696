"""Encoding and grouping (drop-in for src/videotofaces/grouping.py).

classify (grouping.py:50-66) runs its cosine distances / argmin on the GPU
(vtf_cosine_classify).  cluster_faces (grouping.py:92-137) runs KMeans and the three
scores per k on the GPU (videotofaces.kmeans.Grouper, sklearn-faithful); under
torch.distributed the k sweep is sharded across ranks and the per-k labels
and scores are all-gathered.
"""
import math
import os
import os.path as osp
import shutil

import numpy as np
import torch

from . import _native as nat
from .dupes import remove_dupes_overall  # noqa: F401  (re-export like the reference)


def get_encoder_model(style, enc_model, device):
    """grouping.py:19-26 (style coupling kept: anime -> ViT, live -> FaceNet)."""
    if style == 'anime':
        from .encoders.vit import AnimeVIT
        isL = False if enc_model == 'default' else enc_model[-1] == 'l'
        return AnimeVIT(device, isL)
    if style == 'live':
        from .encoders.facenet import FaceNet
        isC = False if enc_model == 'default' else enc_model.split('_')[1] == 'casia'
        return FaceNet(device, isC)
    return 0


def _imread(p):
    try:
        import cv2
        return cv2.imread(p)
    except ImportError:
        from PIL import Image
        return np.asarray(Image.open(p).convert('RGB'))[:, :, ::-1].copy()


def encode_faces(paths, model, bs, area):
    """grouping.py:29-40: batches of images -> model -> concatenated [N, D]."""
    from .utils import crop_to_area
    print('Extracting features from images for grouping')
    x = []
    for bn in range(math.ceil(len(paths) / bs)):
        images = [_imread(p) for p in paths[bs * bn:bs * (bn + 1)]]
        if area:
            images = [crop_to_area(img, area) for img in images]
        x.append(model(images))
    return np.concatenate(x)


def cosine_classify_device(X, R, device=None):
    """classify's distances (grouping.py:51-55): min / first argmin over the reference rows of
    sklearn's cosine_distances(X, R), in sklearn's bits, on `device` (default cuda:0)."""
    dev = nat.require_gpu(device)
    Xd = torch.from_numpy(np.ascontiguousarray(X, np.float32)).to(dev)
    Rd = torch.from_numpy(np.ascontiguousarray(R, np.float32)).to(dev)
    n, d = Xd.shape
    mins = torch.empty(n, dtype=torch.float32, device=dev)
    inds = torch.empty(n, dtype=torch.int64, device=dev)
    nat.check(nat.lib().vtf_cosine_classify(nat.ptr(Xd), n, nat.ptr(Rd), Rd.shape[0], d, nat.ptr(mins), nat.ptr(inds),
                                            nat.stream_ptr(dev)))
    return mins.cpu().numpy(), inds.cpu().numpy()


def cosine_distances_device(X, R, device=None):
    """sklearn.metrics.pairwise.cosine_distances(X, R) (grouping.py:51) in sklearn's bits, [N, C]."""
    dev = nat.require_gpu(device)
    Xd = torch.from_numpy(np.ascontiguousarray(X, np.float32)).to(dev)
    Rd = torch.from_numpy(np.ascontiguousarray(R, np.float32)).to(dev)
    n, d = Xd.shape
    dist = torch.empty((n, Rd.shape[0]), dtype=torch.float32, device=dev)
    nat.check(nat.lib().vtf_cosine_distances_xr(nat.ptr(Xd), n, nat.ptr(Rd), Rd.shape[0], d, nat.ptr(dist),
                                                nat.stream_ptr(dev)))
    return dist.cpu().numpy()


def classify(X, R, classes, thr, log, paths, out_dir, device=None):
    mins, inds = cosine_classify_device(X, R, device)
    if thr and thr != -1:
        inds[mins >= thr] = len(classes)
        classes.append('other')
    if log:
        dist = cosine_distances_device(X, R, device)  # the same bits as the reference's dist
        fnames = [osp.basename(p) for p in paths]
        with open(osp.join(out_dir, 'faces', 'log_classification.csv'), 'w') as f:
            extra = '(other_threshold=%s)' % str(thr) if thr else ''
            f.write('file_name,' + ','.join(['dist_' + c for c in classes if c != 'other']) +
                    ',assigned_to_class' + extra + '\n')
            for i in range(X.shape[0]):
                f.write('%s,' % fnames[i] + ','.join(['%.4f' % d for d in dist[i]]) + ',%s\n' % classes[inds[i]])
    return inds, classes


def cluster_sweep(X, clusters, random_state, grouper=None, device=None, sharded=False, replicated=False):
    """KMeans + (silhouette, CH, DB) for every k in `clusters`, in order -- cluster_faces'
    loops (grouping.py:97-107).  sharded=True (a collective over the default process group:
    every rank passes the same X, which is checked) splits the work across the ranks
     with no cross-rank reduction inside a result, so every number equals the
    one-process result; the results travel by tensor all-gathers (RCCL on GPUs):
      * KMeans fits by k: rank r fits the k at positions i % world == r; labels all-gathered;
      * silhouette by rows: one pass over the distance rows of the rank's row range computes
        silhouette_samples for EVERY k at once (no N x N matrix anywhere); the per-row values
        are all-gathered and averaged in row order as silhouette_score's np.mean does;
      * CH / DB by k, like the fits.
    `grouper` defaults to the device Grouper (videotofaces.kmeans); tests pass a CPU stand-in.
    replicated=True: the caller has already checked that every rank holds X (no digest here)."""
    import torch
    import torch.distributed as dist
    if grouper is None:
        from .kmeans import Grouper
        grouper = Grouper(device)
    g = grouper
    X = np.ascontiguousarray(X, np.float32)
    world = dist.get_world_size() if sharded and dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    if world > 1:
        from .parallel import all_gather_cpu, all_gather_slots, check_replicated
        if not replicated:
            check_replicated(X, 'cluster_sweep')
    prep = g.prepare(X)
    K, n = len(clusters), X.shape[0]
    idx = [i for i in range(K) if i % world == rank]
    fits = {i: np.asarray(g.kmeans(X, clusters[i], random_state=random_state, prep=prep)) for i in idx}
    if world > 1:
        fits = dict(enumerate(all_gather_slots(fits, K, (n,), torch.int64)))
    labels = [fits[i] for i in range(K)]
    lo, hi = n * rank // world, n * (rank + 1) // world
    sil = g.silhouette_sweep(X, labels, lo, hi) if labels else np.zeros((0, 0), np.float32)
    chdb = {i: (g.calinski_harabasz_score(X, labels[i]), g.davies_bouldin_score(X, labels[i])) for i in idx}
    if world > 1:
        if K:  # row-major [rows, K] blocks in rank order -> [K, n]
            sil = all_gather_cpu(torch.from_numpy(np.ascontiguousarray(np.asarray(sil, np.float32).T))).numpy().T
        chdb = dict(enumerate(tuple(float(v) for v in a)
                              for a in all_gather_slots(chdb, K, (2,), torch.float64)))
    scores = [(clusters[i], float(np.mean(sil[i])), float(chdb[i][0]), float(chdb[i][1]))
              for i in range(len(clusters))]
    return labels, scores


def cluster_faces(paths, X, cluster_params, device=None):
    """grouping.py:92-137 with the KMeans / score sweep on the GPU (cluster_sweep); `device`
    (an addition) picks the GPU."""
    clusters, save_all, rstate, log, out_dir = cluster_params
    clusters = [c for c in clusters if c <= len(paths)]
    print('Clustering images into %s groups' % ', '.join([str(cl) for cl in clusters]))
    labels, scores = cluster_sweep(X, clusters, rstate, device=device)
    if log:
        with open(osp.join(out_dir, 'faces', 'log_clustering.csv'), 'w') as f:
            f.write('n_clusters,silhouette_score,calinski_harabasz_score,davies_bouldin_score\n')
            for score in scores:
                f.write('%u,%s,%s,%s\n' % score)
    if not save_all:
        best_k = max(scores, key=lambda x: x[1])[0]
        i = clusters.index(best_k)
        clusters, labels = [clusters[i]], [labels[i]]
        print('The number of groups chosen: %u' % best_k)
    print('Grouped %u images into %s folders:' % (len(paths), '/'.join([str(cl) for cl in clusters])))
    img_dir = osp.dirname(osp.abspath(paths[0]))
    for i in range(len(clusters)):
        k = clusters[i]
        sub = 'G%u' % k if len(clusters) > 1 else ''
        for j in range(k):
            os.makedirs(osp.join(img_dir, sub, str(j)), exist_ok=True)
        for j in range(len(paths)):
            shutil.copyfile(paths[j], osp.join(img_dir, sub, str(labels[i][j]), osp.basename(paths[j])))
        values, counts = np.unique(labels[i], return_counts=True)
        print((sub + ': ' if sub else '') + ', '.join(['%u: %u' % (v, c) for v, c in zip(values, counts)]))
    print()
    for p in paths:
        os.remove(p)
    return clusters, labels, scores


def encode_refs(refs, model):
    """grouping.py:43-47: the first image of every reference class."""
    return model([_imread(ps[0]) for (_, ps) in refs])


def classify_faces(paths, X, model, classif_params, device=None):
    """grouping.py:69-89: classify against reference images, move files into class folders."""
    refs, thr, log, out_dir = classif_params
    classes = [c for (c, _) in refs]
    print('Found %u classes in ref_dir: %s' % (len(classes), ', '.join(classes)))
    print('Extracting features from reference images')
    R = encode_refs(refs, model)
    print('Classifying images')
    inds, classes = classify(X, R, classes, thr, log, paths, out_dir, device or nat.device_of(model))
    img_dir = osp.dirname(osp.abspath(paths[0]))
    for c in classes:
        os.makedirs(osp.join(img_dir, c), exist_ok=True)
    for p, i in zip(paths, inds):
        os.replace(p, osp.join(img_dir, classes[i], osp.basename(p)))
    print('Grouped %u images into %u folders:' % (len(paths), len(classes)))
    for i, c in enumerate(classes):
        print('%s: %u' % (c, np.count_nonzero(inds == i)))
    print()
    return inds, classes
