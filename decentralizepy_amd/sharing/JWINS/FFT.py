"""FFT plugin: top-k over the real-FFT coefficients of the model change, on the MI355X codec.

Drop-in for the reference ``decentralizepy.sharing.JWINS.FFT.FFT``
(``src/decentralizepy/sharing/JWINS/FFT.py``): same constructor keyword arguments
(``alpha, dict_ordered, save_shared, metadata_cap, change_based_selection, save_accumulated,
accumulation, accumulate_averaging_changes, compress, compression_package, compression_class``),
same wire payload ``{alpha, params: complex64[k], indices: int32[k], send_partial: True}`` (full
share: ``{params: complex64[n // 2 + 1]}``) and the same model side effects (complex
``accumulated_changes``, ``shared_parameters_counter`` over the n // 2 + 1 coefficients).

Device path per round:
  pre-step   F(x) = rfft(x) and F(x - x0) (dpz_rfft: the native mixed-radix kernels; the
             difference by dpz_elementwise)
  encode     |change| after the accumulation step (dpz_cplx_key), the shared top-k kernels on that
             fp32 key (counter fused), complex values gathered from F(x) with the rewind fused
             (dpz_cplx_gather)                                              (FFT.py:132-211)
  averaging  the batched replace + Metro-Hastings fold over the interleaved (re, im) view of the
             coefficients (complex entries as float pairs), then irfft      (FFT.py:252-302)

Parity is a tolerance parity: an fp32 FFT rounds differently from torch's CPU pocketfft;
the selection, the fold order and the bookkeeping are the reference's.
"""
import numpy as np
import torch

from ... import codec
from ..._device import to_host
from ...utils import identity
from ..PartialModel import PartialModel


class FFT(PartialModel):
    """This class implements the fft version of model sharing."""

    def __init__(self, rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                 alpha=1.0, dict_ordered=True, save_shared=False, metadata_cap=1.0,
                 change_based_selection=True, save_accumulated="", accumulation=False,
                 accumulate_averaging_changes=False, compress=False, compression_package=None,
                 compression_class=None):
        super().__init__(rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                         alpha, dict_ordered, save_shared, metadata_cap, accumulation,
                         save_accumulated, identity, accumulate_averaging_changes, compress,
                         compression_package, compression_class)
        self.change_based_selection = change_based_selection
        if self.accumulation:  # zeros_like(rfft(init)): complex (reference PartialModel.py:116-119)
            self.model.accumulated_changes = torch.zeros(self.transformed_len,
                                                         dtype=torch.complex64, device=self.device)
        self._diff = None

    # ---- PartialModel hooks --------------------------------------------------------------------
    def _check_transformer(self):
        pass

    def _transformed_len(self):
        return self.number_of_params // 2 + 1

    def _rfft(self, x):
        return codec.rfft(x, workspace=self.workspace)

    def _transform_pre_step(self, x):
        """(rfft(x), rfft(x - init)) (reference PartialModel.py:311-320 with T = rfft)."""
        if self._diff is None or self._diff.numel() != x.numel():
            self._diff = torch.empty_like(x)
        codec.elementwise(codec.DPZ_EW_SUB, x, self.init_model, out=self._diff)
        return self._rfft(x), self._rfft(self._diff)

    def _encode(self, k):
        """reference FFT.py:132-156 + PartialModel.py:321-329 on complex coefficients; returns
        device (idx int32[k], vals complex64[k])."""
        acc = self.model.accumulated_changes if self.accumulation else None
        mode = self._acc_mode()
        fx, change = self.pre_share_model_transformed, self._change_dev
        if self.change_based_selection:
            key = codec.cplx_key(change, acc, mode)
        else:
            if mode == codec.DPZ_ACC_ACCUMULATE:  # the _pre_step bookkeeping still happens
                codec.cplx_key(change, acc, mode)
            key = codec.cplx_key(fx)
        idx, _ = codec.topk_encode(key, k, idx_out=self._ring_slot(k), workspace=self.workspace)
        self._ring_commit(idx)
        vals = codec.cplx_gather(fx, idx, acc=acc)
        return idx, vals

    def _accumulate_change(self, new, prev):
        """acc += rfft(new - prev) (reference PartialModel.py:346-349 with T = rfft)."""
        if self._diff is None or self._diff.numel() != new.numel():
            self._diff = torch.empty_like(new)
        codec.elementwise(codec.DPZ_EW_SUB, new, prev, out=self._diff)
        d = self._rfft(self._diff)
        codec.elementwise(codec.DPZ_EW_ADD, self.model.accumulated_changes.view(torch.float32),
                          d.view(torch.float32),
                          out=self.model.accumulated_changes.view(torch.float32))

    def _zero_accumulation(self):
        if getattr(self.model, "accumulated_changes", None) is not None:
            self.model.accumulated_changes.zero_()

    # ---- wire format ------------------------------------------------------------------------------
    def compress_data(self, data, idx_dev=None, val_dev=None):
        """Indices may take the device index codec; complex values go through the compressor's
        host ``compress_float`` as in the reference (FFT.py:211 -> PartialModel.py:147-154).
        Only a pass-through value leg (Compression / Elias: ``compress_float`` is the identity)
        can carry complex64: the float codecs (fpzip-class, LZ4, fp16) are fp32 codecs, and the
        reference's fail on or silently reinterpret complex input (fpzip.compress rejects it,
        EliasFpzip.py:34; Lz4Wrapper decodes the bytes as float32, Lz4Wrapper.py:94-98), so this
        raises instead of corrupting the average."""
        from ...compression.Compression import Compression
        if (self.compress and "params" in data and np.iscomplexobj(data["params"])
                and type(self.compressor).compress_float is not Compression.compress_float):
            raise NotImplementedError(
                f"FFT: complex64 payload values cannot go through "
                f"{type(self.compressor).__name__}.compress_float (an fp32 codec); use "
                "compression_class Elias (indices only) or compress = False")
        return super().compress_data(data, idx_dev=idx_dev, val_dev=None)

    def _full_share(self):
        """alpha >= metadata_cap: every coefficient (reference FFT.py:169-176)."""
        m = dict()
        m["params"] = to_host(self.pre_share_model_transformed, self.staging, "coeffs")
        self._zero_accumulation()
        return self.compress_data(m)

    def _message(self, indices, params):
        m = dict()  # key order of reference FFT.py:206-209
        m["alpha"] = self.alpha
        m["params"] = params
        m["indices"] = indices.astype(np.int32)
        m["send_partial"] = True
        return m

    def serialized_model(self):
        """reference FFT.py:158-211"""
        if self.alpha >= self.metadata_cap:
            return self._full_share()
        return PartialModel.serialized_model(self)

    def deserialized_model(self, m):
        """reference FFT.py:213-250: tensors of the payload, no merging."""
        m = self.decompress_data(m)
        ret = dict()
        if "send_partial" not in m:  # the reference falls through to m["indices"]: KeyError
            ret["params"] = torch.tensor(m["params"])
        with torch.no_grad():
            if not self.dict_ordered:
                raise NotImplementedError
            ret["indices"] = torch.tensor(m["indices"], dtype=torch.long)
            ret["params"] = torch.tensor(m["params"])
            ret["send_partial"] = True
        return ret

    # ---- receive side ---------------------------------------------------------------------------
    def _device_payload(self, data):
        """Complex payload -> (float-pair idx int32[2k] or None, fp32 view of the values)."""
        vals = self._h2d(data["params"], np.complex64, "vals")
        idx = data["indices"]  # a full payload raises KeyError, as in the reference (FFT.py:234)
        return codec.cplx_pair_indices(self._h2d(idx, np.int32, "idx")), vals.view(torch.float32)

    def _averaging(self, peer_deques):
        """reference FFT.py:252-302: Metro-Hastings fold of the coefficients, then irfft."""
        with torch.no_grad():
            payloads, degrees = self._pop_payloads(peer_deques)
            weights = [1 / (max(len(peer_deques), d) + 1) for d in degrees]
            weight_total = 0
            for w in weights:
                weight_total += w
            local = self._local_flat_device()
            if local is self.pre_share_model and self.pre_share_model_transformed is not None:
                flat_fft = self.pre_share_model_transformed
            else:
                flat_fft = self._rfft(local)
            total = codec.decode_average(flat_fft.view(torch.float32), payloads, weights,
                                         1 - weight_total, workspace=self.workspace)
            n_out = 2 * (self.transformed_len - 1)  # irfft's default length
            if n_out != self.number_of_params:
                raise RuntimeError(
                    f"irfft returns {n_out} values for a model of {self.number_of_params} "
                    "parameters (odd sizes fail in the reference's reshape as well)")
            out = codec.irfft(total.view(torch.complex64), n_out, workspace=self.workspace)
            self._load_flat(out)
        self._post_step()
        self.communication_round += 1

    def _averaging_server(self, peer_deques):
        """The reference FFT inherits Sharing._averaging_server, which loads the frequency-domain
        payload dict as a state_dict and fails in load_state_dict; so does this one, before
        touching any state."""
        raise RuntimeError("Error(s) in loading state_dict: the FFT plugin has no server average "
                           "(reference sharing/Sharing.py:200-229 on FFT payloads)")
