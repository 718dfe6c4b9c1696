"""Encoding and grouping (drop-in for src/videotofaces/grouping.py).

classify (grouping.py:50-66) runs its cosine distances / argmin on the GPU
(vtf_cosine_classify).  cluster_faces keeps sklearn's KMeans and scores on the host (the
reference's own dependency, sklearn 1.7.2 here); the K-means / silhouette kernels are
the next §8 rows.
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


def cosine_classify_device(X, R):
    dev = torch.device('cuda:0')
    Xd = torch.from_numpy(np.ascontiguousarray(X, np.float32)).to(dev)
    Rd = torch.from_numpy(np.ascontiguousarray(R, np.float32)).to(dev)
    n, d = Xd.shape
    mins = torch.empty(n, dtype=torch.float32, device=dev)
    inds = torch.empty(n, dtype=torch.int64, device=dev)
    nat.check(nat.lib().vtf_cosine_classify(nat.ptr(Xd), n, nat.ptr(Rd), Rd.shape[0], d, nat.ptr(mins), nat.ptr(inds),
                                            nat.stream_ptr(dev)))
    return mins.cpu().numpy(), inds.cpu().numpy()


def classify(X, R, classes, thr, log, paths, out_dir):
    mins, inds = cosine_classify_device(X, R)
    if thr and thr != -1:
        inds[mins >= thr] = len(classes)
        classes.append('other')
    if log:
        import sklearn.metrics
        dist = sklearn.metrics.pairwise.cosine_distances(X, R)
        fnames = [osp.basename(p) for p in paths]
        with open(osp.join(out_dir, 'faces', 'log_classification.csv'), 'w') as f:
            extra = '(other_threshold=%s)' % str(thr) if thr else ''
            f.write('file_name,' + ','.join(['dist_' + c for c in classes if c != 'other']) +
                    ',assigned_to_class' + extra + '\n')
            for i in range(X.shape[0]):
                f.write('%s,' % fnames[i] + ','.join(['%.4f' % d for d in dist[i]]) + ',%s\n' % classes[inds[i]])
    return inds, classes


def cluster_faces(paths, X, cluster_params):
    """grouping.py:92-137 (sklearn KMeans + silhouette / CH / DB on the host)."""
    import sklearn.cluster
    import sklearn.metrics
    clusters, save_all, rstate, log, out_dir = cluster_params
    clusters = [c for c in clusters if c <= len(paths)]
    print('Clustering images into %s groups' % ', '.join([str(cl) for cl in clusters]))
    labels = [sklearn.cluster.KMeans(n_clusters=k, random_state=rstate, n_init='auto').fit(X).labels_ for k in clusters]
    scores = []
    for i in range(len(clusters)):
        scores.append((clusters[i], sklearn.metrics.silhouette_score(X, labels[i]),
                       sklearn.metrics.calinski_harabasz_score(X, labels[i]),
                       sklearn.metrics.davies_bouldin_score(X, labels[i])))
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
    img_dir = osp.dirname(osp.abspath(paths[0]))
    for i in range(len(clusters)):
        k = clusters[i]
        sub = 'G%u' % k if len(clusters) > 1 else ''
        for j in range(k):
            os.makedirs(osp.join(img_dir, sub, str(j)), exist_ok=True)
        for j in range(len(paths)):
            shutil.copyfile(paths[j], osp.join(img_dir, sub, str(labels[i][j]), osp.basename(paths[j])))
    for p in paths:
        os.remove(p)
    return clusters, labels, scores
