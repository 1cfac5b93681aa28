"""Wavelet plugin: top-k in the sym2 wavelet domain, on the MI355X codec.

Drop-in for the reference ``decentralizepy.sharing.JWINS.Wavelet.Wavelet``
(``src/decentralizepy/sharing/JWINS/Wavelet.py``): same constructor keyword arguments
(``alpha, dict_ordered, save_shared, metadata_cap, wavelet, level, change_based_selection,
save_accumulated, accumulation, accumulate_averaging_changes, compress, compression_package,
compression_class``), same wire payloads and the same model side effects.

Device path per round (all HIP kernels, fp32, pywt-1.1.1-exact summation order):
  pre-step   W(x) and W(x - x0) in ONE multilevel DWT launch (reference Wavelet.py:30-32 called
             twice from PartialModel.py:317-320)
  encode     top-k on |W(x - x0)| (+ accumulation), values gathered from W(x) (Wavelet.py:142-231);
             with accumulate_averaging_changes the counter / rewind bookkeeping is coalesced
             (bit-sliced counter, selection mask; dpz_topk_encode_sliced)
  averaging  one batched replace+fold over all payloads in the wavelet domain, then one
             multilevel IDWT launch (Wavelet.py:269-329)
  post-step  acc += W(x_new - prev) as one accumulating DWT launch (PartialModel.py:346-349),
             applying the encode's deferred rewind as it goes (dpz_dwt_sym2_rewind)

Fused device kernels run ``wavelet="sym2"`` with ``level <= 4`` (every shipped JWINS config,
e.g. tutorial/JWINS/config.ini) and the reference's default ``wavelet="haar"`` with
``level <= 8``; every other pywt discrete wavelet with an even filter length <= 64 (db1-32,
sym2-20, coif1-10, bior / rbio, dmey) and levels to 8 runs the generic-filter kernels
(dpz_dwt_generic / dpz_idwt_generic), bit-exact with PyWavelets 1.1.1 as well.  A level at which
an input would be shorter than the filter (pywt's multi-reflection case) raises
NotImplementedError, as do names pywt does not know.
"""
import numpy as np
import torch

from ... import codec
from ..._device import DeviceAccumulator, SlicedCounter, to_host
from ...utils import identity
from ..PartialModel import PartialModel

MAX_LEVEL = 8


def coeff_slices(n, level, wavelet="sym2"):
    """``pywt.coeffs_to_array`` slices of a 1-D ``wavedec`` (array layout [cA_L, cD_L..cD_1]);
    level lengths floor((len + filter_len - 1) / 2) (pywt.dwt_coeff_len, mode symmetric)."""
    f = codec.filter_len(wavelet)
    lens = [int(n)]
    for _ in range(level):
        lens.append((lens[-1] + f - 1) // 2)
    slices = [slice(0, lens[level])]
    pos = lens[level]
    for lvl in range(level, 0, -1):
        slices.append({"d": (slice(pos, pos + lens[lvl]),)})
        pos += lens[lvl]
    return slices, pos


class Wavelet(PartialModel):
    """This class implements the wavelet version of model sharing."""

    def __init__(self, rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                 alpha=1.0, dict_ordered=True, save_shared=False, metadata_cap=1.0,
                 wavelet="haar", level=4, change_based_selection=True, save_accumulated="",
                 accumulation=False, accumulate_averaging_changes=False, compress=False,
                 compression_package=None, compression_class=None):
        self.wavelet = wavelet
        self.level = int(level)
        if wavelet not in codec.wavelet_names():
            raise NotImplementedError(
                f"wavelet '{wavelet}': the device DWT kernels implement sym2, haar and the pywt "
                f"discrete wavelets with filter length <= 64 (codec.wavelet_names())")
        if not 1 <= self.level <= MAX_LEVEL:
            raise NotImplementedError(f"the device DWT kernels implement levels 1..{MAX_LEVEL}")
        super().__init__(rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                         alpha, dict_ordered, save_shared, metadata_cap, accumulation,
                         save_accumulated, identity, accumulate_averaging_changes, compress,
                         compression_package, compression_class)
        self.change_based_selection = change_based_selection
        slices, m = coeff_slices(self.number_of_params, self.level, self.wavelet)
        self.wt_shape = (m,)
        self.coeff_slices = slices
        # accumulation with accumulate_averaging_changes (the JWINS tutorial config): the encode's
        # bookkeeping in coalesced form — the counter as bit planes, the rewind deferred to the
        # post-step's accumulating DWT, which rewrites the accumulator anyway
        # (dpz_topk_encode_sliced, dpz_dwt_sym2_rewind)
        self._sliced = bool(self.accumulation and self.accumulate_averaging_changes)
        if self._sliced:
            nw = codec.mask_words(self.transformed_len)
            self._planes = torch.zeros(32 * nw, dtype=torch.int32, device=self.device)
            self._sel_mask = torch.zeros(nw, dtype=torch.int32, device=self.device)
            self._counter = None
            self._ring = None  # the sliced planes replace the int32 counter and its ring
            self.model.shared_parameters_counter = SlicedCounter(self._planes,
                                                                 self.transformed_len)
            self.model.accumulated_changes = DeviceAccumulator(self.model.accumulated_changes)

    # ---- PartialModel hooks --------------------------------------------------------------------
    def _check_transformer(self):
        pass

    def _transformed_len(self):
        return codec.wavedec_len(self.number_of_params, self.level, self.wavelet)

    def _transform_pre_step(self, x):
        """W(x), W(x - init) in one DWT launch."""
        return codec.wavedec(x, self.level, x0=self.init_model, wavelet=self.wavelet)

    def _encode(self, k):
        acc = self._acc()
        wx, wc = self.pre_share_model_transformed, self._change_dev
        if self._sliced:
            # counter += 1 on the bit planes, rewind left pending (applied by _accumulate_change)
            if self.change_based_selection:
                idx, val = codec.topk_encode_sliced(wc, k, self._sel_mask, self._planes, acc=acc,
                                                    acc_mode=codec.DPZ_ACC_ADD, vals_src=wx,
                                                    workspace=self.workspace)
            else:
                idx, val = codec.topk_encode_sliced(wx, k, self._sel_mask, self._planes,
                                                    vals_src=wx, workspace=self.workspace)
            self.model.accumulated_changes.pending = self._sel_mask
            return idx, val
        if self.change_based_selection:
            idx, val = codec.topk_encode(wc, k, acc=acc, acc_mode=self._acc_mode(), vals_src=wx,
                                         idx_out=self._ring_slot(k), workspace=self.workspace)
            self._ring_commit(idx)
            return idx, val
        # selection on |W(x)|; the accumulation bookkeeping of _pre_step and the rewind still apply
        if self._acc_mode() == codec.DPZ_ACC_ACCUMULATE:
            codec.topk_encode(wc, 0, acc=acc, acc_mode=codec.DPZ_ACC_ACCUMULATE,
                              workspace=self.workspace)
        idx, val = codec.topk_encode(wx, k, vals_src=wx, idx_out=self._ring_slot(k),
                                     workspace=self.workspace)
        self._ring_commit(idx)
        if acc is not None:
            codec.scatter_fill(acc, idx, 0.0)
        return idx, val

    def _full_share(self):
        """alpha >= metadata_cap: all coefficients W(x) (reference Wavelet.py:185-192).  With a
        device float compressor the coefficients are coded where they are (no D2H of the raw
        4M bytes and H2D back into the compressor)."""
        m = dict()
        wx = self.pre_share_model_transformed
        dev_codec = self.compress and hasattr(getattr(self, "compressor", None),
                                              "compress_float_device")
        m["params"] = None if dev_codec else to_host(wx, self.staging, "coeffs")
        self._zero_accumulation()
        if dev_codec:
            return self.compress_data(m, val_dev=wx)
        return self.compress_data(m)

    def _message(self, indices, params):
        m = dict()  # key order of reference Wavelet.py:223-229
        m["alpha"] = self.alpha
        m["params"] = params
        m["indices"] = indices.astype(np.int32)
        m["send_partial"] = True
        return m

    def _accumulate_change(self, new, prev):
        """acc += W(new - prev) (reference PartialModel.py:346-349 with T = wavelet); a rewind the
        encode left pending is applied by the same pass (acc = (selected ? 0 : acc) + W)."""
        a = self.model.accumulated_changes
        if isinstance(a, DeviceAccumulator):
            if a.pending is not None:
                codec.wavedec(new, self.level, x0=prev, want_x=False, coeffs_diff=a.device_tensor,
                              accumulate=True, wavelet=self.wavelet, rewind_mask=a.pending)
                a.pending = None
                return
            a = a.device_tensor
        codec.wavedec(new, self.level, x0=prev, want_x=False, coeffs_diff=a, accumulate=True,
                      wavelet=self.wavelet)

    # ---- receive side -------------------------------------------------------------------------
    def deserialized_model(self, m):
        """reference Wavelet.py:233-267: tensors of the payload, no merging."""
        m = self.decompress_data(m)
        ret = dict()
        if "send_partial" not in m:
            ret["params"] = torch.tensor(m["params"])
            return ret
        with torch.no_grad():
            if not self.dict_ordered:
                raise NotImplementedError
            ret["indices"] = torch.tensor(m["indices"], dtype=torch.long)
            ret["params"] = torch.tensor(m["params"])
            ret["send_partial"] = True
        return ret

    def _coeff_fold_and_reconstruct(self, peer_deques, server):
        payloads, degrees = self._pop_payloads(peer_deques)
        if server:
            weights, w_self = [1 / len(peer_deques)] * len(payloads), None
        else:
            weights = [1 / (max(len(peer_deques), d) + 1) for d in degrees]
            weight_total = 0
            for w in weights:
                weight_total += w
            w_self = 1 - weight_total
        total = self._fold(self.pre_share_model_transformed, payloads, weights, w_self)
        return codec.waverec(total, self.number_of_params, self.level, wavelet=self.wavelet)

    def _averaging(self, peer_deques):
        """reference Wavelet.py:269-329: fold in the wavelet domain, then waverec."""
        with torch.no_grad():
            out = self._coeff_fold_and_reconstruct(peer_deques, server=False)
            self._load_flat(out)
        self._post_step()
        self.communication_round += 1

    def _averaging_server(self, peer_deques):
        """reference Wavelet.py:331-385"""
        with torch.no_grad():
            out = self._coeff_fold_and_reconstruct(peer_deques, server=True)
            self._load_flat(out)
        self._post_step()
        self.communication_round += 1

    def serialized_model(self):
        """reference Wavelet.py:174-231"""
        if self.alpha >= self.metadata_cap:
            return self._full_share()
        return PartialModel.serialized_model(self)

