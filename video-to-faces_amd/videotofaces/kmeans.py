"""K-means and cluster scores on MI355X: the sklearn calls of cluster_faces
(src/videotofaces/grouping.py:97-107) on device.

Mirrors scikit-learn 1.7 (the reference's unpinned dependency, requirements.txt:5):
  KMeans(n_clusters=k, random_state=rs, n_init='auto').fit(X).labels_
      sklearn/cluster/_kmeans.py: fit 1428-1545 (mean-centring, tol = mean(var) * 1e-4,
      n_init 'auto' -> 1 for k-means++), _kmeans_plusplus 174-276, _kmeans_single_lloyd 620-745;
      _k_means_lloyd.pyx lloyd_iter_chunked_dense; _k_means_common.pyx relocation / averaging.
  silhouette_score, calinski_harabasz_score, davies_bouldin_score
      sklearn/metrics/cluster/_unsupervised.py.
The scalar control flow (RandomState draws, searchsorted over the float64 cumsum, argmin of
candidate potentials, convergence tests) runs here on host numpy exactly as sklearn writes
it; every pass over X (centring, k-means++ distance rows, E/M steps, the silhouette sweep over
the distance rows -- never an N x N matrix -- and the cluster statistics) is a libvtf_hip.so
kernel.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat


class Grouper:
    """Device-side grouping math for one GPU (vtf_group_*)."""

    def __init__(self, device=None):
        self.device = nat.require_gpu(device)
        h = ctypes.c_void_p()
        nat.check(nat.lib().vtf_group_create(self.device.index or 0, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h and nat._LIB is not None:
            nat._LIB.vtf_group_destroy(h)
            self._h = None

    def _bind(self):
        nat.check(nat.lib().vtf_group_set_stream(self._h, nat.stream_ptr(self.device)))

    def _dev(self, X):
        X = torch.as_tensor(X)
        if X.dtype != torch.float32:
            X = X.float()
        return X.to(self.device).contiguous()

    # ------------------------------------------------------------------ KMeans
    def prepare(self, X):
        """Centred X, per-column mean and variance (shared by every k of a sweep)."""
        X = self._dev(X)
        N, D = X.shape
        Xc = torch.empty_like(X)
        mean = torch.empty(D, dtype=torch.float32, device=self.device)
        var = torch.empty(D, dtype=torch.float32, device=self.device)
        self._bind()
        nat.check(nat.lib().vtf_colstats(self._h, nat.ptr(X), N, D, nat.ptr(Xc), nat.ptr(mean), nat.ptr(var)))
        return {'X': X, 'Xc': Xc, 'var': var.cpu().numpy()}

    def _sqdist_rows(self, Xc, ids):
        ids = np.ascontiguousarray(np.asarray(ids, np.int64).reshape(-1))
        N, D = Xc.shape
        self._bind()
        out = torch.empty((ids.size, N), dtype=torch.float32, device=self.device)
        nat.check(nat.lib().vtf_sqdist_rows(self._h, nat.ptr(Xc), N, D, ids.ctypes.data, ids.size, nat.ptr(out)))
        return out.cpu().numpy()

    def _kmeans_plusplus(self, Xc, n_clusters, sample_weight, random_state):
        """_kmeans_plusplus (_kmeans.py:174-276) with the distance rows on device."""
        n_samples = Xc.shape[0]
        n_local_trials = 2 + int(np.log(n_clusters))
        center_id = random_state.choice(n_samples, p=sample_weight / sample_weight.sum())
        indices = np.full(n_clusters, -1, dtype=int)
        indices[0] = center_id
        closest_dist_sq = self._sqdist_rows(Xc, [center_id])
        current_pot = closest_dist_sq @ sample_weight
        for c in range(1, n_clusters):
            rand_vals = random_state.uniform(size=n_local_trials) * current_pot
            candidate_ids = np.searchsorted(np.cumsum(sample_weight * closest_dist_sq, dtype=np.float64), rand_vals)
            np.clip(candidate_ids, None, closest_dist_sq.size - 1, out=candidate_ids)
            distance_to_candidates = self._sqdist_rows(Xc, candidate_ids)
            np.minimum(closest_dist_sq, distance_to_candidates, out=distance_to_candidates)
            candidates_pot = distance_to_candidates @ sample_weight.reshape(-1, 1)
            best_candidate = np.argmin(candidates_pot)
            current_pot = candidates_pot[best_candidate]
            closest_dist_sq = distance_to_candidates[best_candidate]
            indices[c] = candidate_ids[best_candidate]
        return indices

    # ---- device primitives (one kernel pass each)
    def _step(self, Xc, centers, labels, k, update_centers):
        """E-step (+ M-step sums): returns (sums, weights as host np.float32, changed)."""
        N, D = Xc.shape
        self._bind()
        L = nat.lib()
        changed = ctypes.c_int64(0)
        if not update_centers:
            nat.check(L.vtf_kmeans_step(self._h, nat.ptr(Xc), N, D, nat.ptr(centers), k, nat.ptr(labels), None, None,
                                        ctypes.byref(changed)))
            return None, None, changed.value
        sums = torch.empty((k, D), dtype=torch.float32, device=self.device)
        w = torch.empty(k, dtype=torch.float32, device=self.device)
        nat.check(L.vtf_kmeans_step(self._h, nat.ptr(Xc), N, D, nat.ptr(centers), k, nat.ptr(labels), nat.ptr(sums),
                                    nat.ptr(w), ctypes.byref(changed)))
        return sums, w.cpu().numpy(), changed.value

    def _average(self, sums, w, centers_old):
        """_average_centers + _center_shift in place on sums; returns host shift."""
        k, D = sums.shape
        dw = torch.from_numpy(np.ascontiguousarray(w)).to(self.device)
        shift = torch.empty(k, dtype=torch.float32, device=self.device)
        nat.check(nat.lib().vtf_kmeans_average(self._h, nat.ptr(sums), nat.ptr(dw), nat.ptr(centers_old), k, D,
                                               nat.ptr(shift)))
        return shift.cpu().numpy()

    def _center_dist(self, Xc, centers, labels):
        N, D = Xc.shape
        dist = torch.empty(N, dtype=torch.float32, device=self.device)
        nat.check(nat.lib().vtf_center_dist(self._h, nat.ptr(Xc), N, D, nat.ptr(centers), nat.ptr(labels),
                                            nat.ptr(dist)))
        return dist.cpu().numpy()

    def _rows(self, Xc, idx):
        return Xc[torch.from_numpy(np.asarray(idx, np.int64)).to(self.device)].contiguous()

    def _to_host(self, t):
        return t.cpu().numpy()

    def _from_host(self, a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def _new_labels(self, N):
        return torch.full((N,), -1, dtype=torch.int32, device=self.device)

    # ---- sklearn control flow
    def _lloyd_iter(self, Xc, centers, labels, k, update_centers=True):
        """lloyd_iter_chunked_dense (_k_means_lloyd.pyx) -> (new centers, shift, changed)."""
        sums, w, changed = self._step(Xc, centers, labels, k, update_centers)
        if not update_centers:
            return None, None, changed
        if np.any(w == 0):
            sums, w = self._relocate_empty(Xc, centers, sums, w, labels)
        shift = self._average(sums, w, centers)
        return sums, shift, changed

    def _relocate_empty(self, Xc, centers_old, sums, weight_in_clusters, labels):
        """_relocate_empty_clusters_dense (_k_means_common.pyx:167-211); sample weights 1."""
        empty_clusters = np.where(np.equal(weight_in_clusters, 0))[0].astype(np.int32)
        n_empty = empty_clusters.shape[0]
        distances = self._center_dist(Xc, centers_old, labels)
        w = weight_in_clusters.copy()
        if np.max(distances) == 0:
            return sums, w
        far_from_centers = np.argpartition(distances, -n_empty)[:-n_empty - 1:-1].astype(np.int32)
        cn = self._to_host(sums).copy()
        lab = self._to_host(labels)
        xs = self._to_host(self._rows(Xc, far_from_centers[:n_empty]))
        for idx in range(n_empty):
            new_cluster_id = empty_clusters[idx]
            far_idx = far_from_centers[idx]
            weight = np.float32(1.0)
            old_cluster_id = lab[far_idx]
            cn[old_cluster_id] -= xs[idx] * weight
            cn[new_cluster_id] = xs[idx] * weight
            w[new_cluster_id] = weight
            w[old_cluster_id] -= weight
        return self._from_host(cn), w

    def kmeans(self, X, n_clusters, random_state=0, tol=1e-4, max_iter=300, prep=None):
        """KMeans(n_clusters, random_state=random_state, n_init='auto').fit(X).labels_ (int32)."""
        p = prep or self.prepare(X)
        Xc = p['Xc']
        N = Xc.shape[0]
        if n_clusters > N:
            raise ValueError('n_samples=%d should be >= n_clusters=%d.' % (N, n_clusters))
        if n_clusters > 64:
            # vtf_kmeans_step keeps a block's distances to every center in LDS (csrc/kmeans.hip)
            raise ValueError('KMeans on the device supports at most 64 clusters (n_clusters=%d); the '
                             'reference sweeps k = 2..16 (grouping.py:97)' % n_clusters)
        tol_abs = np.mean(p['var']) * tol                      # _tolerance (_kmeans.py:279-287)
        rs = np.random.RandomState(random_state) if not isinstance(random_state, np.random.RandomState) \
            else random_state
        sample_weight = np.ones(N, dtype=np.float32)
        idx = self._kmeans_plusplus(Xc, n_clusters, sample_weight, rs)
        centers = self._rows(Xc, idx)
        labels = self._new_labels(N)
        strict = False
        for _ in range(max_iter):
            centers_new, center_shift, changed = self._lloyd_iter(Xc, centers, labels, n_clusters)
            centers = centers_new
            if changed == 0:
                strict = True
                break
            if (center_shift ** 2).sum() <= tol_abs:
                break
        if not strict:
            self._lloyd_iter(Xc, centers, labels, n_clusters, update_centers=False)
        return np.asarray(self._to_host(labels), np.int32)

    # ------------------------------------------------------------------ scores
    @staticmethod
    def _encode(labels):
        """LabelEncoder().fit_transform + np.bincount (silhouette_samples prologue)."""
        classes, enc = np.unique(np.asarray(labels), return_inverse=True)
        n = enc.shape[0]
        if not 1 < len(classes) < n:
            raise ValueError('Number of labels is %d. Valid values are 2 to n_samples - 1 (inclusive)'
                             % len(classes))
        return enc.astype(np.int32), np.bincount(enc).astype(np.int64), len(classes)

    def silhouette_sweep(self, X, label_sets, lo=0, hi=None):
        """silhouette_samples(X, labels) for every label set, rows [lo, hi) -> float32 [M, hi-lo]
        (vtf_silhouette_sweep: one pass over the distance rows per <= 160 clusters of label
        sets, no N x N matrix)."""
        X = self._dev(X)
        N, D = X.shape
        hi = N if hi is None else hi
        out = np.zeros((len(label_sets), hi - lo), np.float32)
        enc = [self._encode(lb) for lb in label_sets]
        i = 0
        while i < len(enc):
            j, c = i, 0
            while j < len(enc) and j - i < 32 and c + enc[j][2] <= 160:
                c += enc[j][2]
                j += 1
            if j == i:
                raise ValueError('silhouette: %d labels (at most 160 per label set here)' % enc[i][2])
            lab = np.stack([e[0] for e in enc[i:j]]).astype(np.uint8)
            ks = np.ascontiguousarray([e[2] for e in enc[i:j]], np.int32)
            freq = np.ascontiguousarray(np.concatenate([e[1] for e in enc[i:j]]), np.int64)
            dl = torch.from_numpy(lab).to(self.device)
            sil = torch.empty((j - i, hi - lo), dtype=torch.float32, device=self.device)
            self._bind()
            nat.check(nat.lib().vtf_silhouette_sweep(self._h, nat.ptr(X), N, D, lo, hi, nat.ptr(dl), j - i,
                                                     ks.ctypes.data, freq.ctypes.data, nat.ptr(sil)))
            out[i:j] = sil.cpu().numpy()
            i = j
        return out

    def silhouette_samples(self, X, labels):
        return self.silhouette_sweep(X, [labels])[0]

    def silhouette_score(self, X, labels):
        return float(np.mean(self.silhouette_samples(X, labels)))

    def _cluster_stats(self, X, labels):
        X = self._dev(X)
        enc, _, k = self._encode(labels)
        N, D = X.shape
        dl = torch.from_numpy(enc).to(self.device)
        sums = torch.empty((k, D), dtype=torch.float64, device=self.device)
        sqn = torch.empty(k, dtype=torch.float64, device=self.device)
        cnt = torch.empty(k, dtype=torch.int64, device=self.device)
        self._bind()
        nat.check(nat.lib().vtf_cluster_sums(self._h, nat.ptr(X), N, D, nat.ptr(dl), k, nat.ptr(sums), nat.ptr(sqn),
                                             nat.ptr(cnt)))
        return X, dl, k, sums.cpu().numpy(), sqn.cpu().numpy(), cnt.cpu().numpy()

    def calinski_harabasz_score(self, X, labels):
        """calinski_harabasz_score (_unsupervised.py:325-367), float64 statistics."""
        X, _, k, sums, sqn, cnt = self._cluster_stats(X, labels)
        n = X.shape[0]
        mean = sums.sum(0) / n
        cent = sums / cnt[:, None]
        extra = float((cnt * ((cent - mean) ** 2).sum(1)).sum())
        intra = float((sqn - cnt * (cent ** 2).sum(1)).sum())
        return 1.0 if intra == 0.0 else extra * (n - k) / (intra * (k - 1.0))

    def davies_bouldin_score(self, X, labels):
        """davies_bouldin_score (_unsupervised.py:396-463), float64 statistics."""
        X, dl, k, sums, _, cnt = self._cluster_stats(X, labels)
        N, D = X.shape
        cent = sums / cnt[:, None]
        dc = torch.from_numpy(np.ascontiguousarray(cent)).to(self.device)
        dsum = torch.empty(k, dtype=torch.float64, device=self.device)
        nat.check(nat.lib().vtf_cluster_dist(self._h, nat.ptr(X), N, D, nat.ptr(dl), k, nat.ptr(dc), nat.ptr(dsum)))
        intra = dsum.cpu().numpy() / cnt
        cd = np.sqrt(np.maximum(((cent[:, None, :] - cent[None, :, :]) ** 2).sum(-1), 0))
        if np.allclose(intra, 0) or np.allclose(cd, 0):
            return 0.0
        cd[cd == 0] = np.inf
        comb = intra[:, None] + intra
        return float(np.mean(np.max(comb / cd, axis=1)))
