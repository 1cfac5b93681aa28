"""STC plugin (sparse top-k with residual error feedback) on the MI355X codec.

Drop-in for the reference ``decentralizepy.sharing.STC.STC`` (``src/decentralizepy/sharing/
STC.py``, the paper's Algorithm 2): same constructor keyword arguments (``alpha, dict_ordered,
change_transformer, compress, compression_package, compression_class, float_precision``), same
methods (``get_data_to_send``, ``server_broadcast``, ``process_received``, ``_averaging_server``,
``serialized_model``, ``deserialized_model``, ``_pre_step``, ``_post_step``), same wire dicts
(``{alpha, indices:int32[k], params:fp32[k]}`` + ``iteration``) and the same model side effects.

Device path (all HIP kernels, fp32, bit-exact with the reference's operation order):
  get_data_to_send   ONE top-k launch sequence with the residual buffer as the accumulator:
                     residuals += flat - prev (= model_change), top-k of |model_change|, values
                     model_change[idx], residuals[idx] = 0 (= model_change - T, STC.py:305-315)
  _averaging_server  one zero-based batched fold total = sum (1/n) T_i, then
                     model_change = residuals + total (STC.py:333-362)
  server_broadcast   top-k of model_change, residuals = model_change with zeros at idx,
                     process_received of its own message (STC.py:317-331)
  process_received   model = flat + T in one add-scatter launch (STC.py:270-303)
State kept in HBM across rounds: prev_model, residuals, model_change (N fp32 each).
"""
import logging

import numpy as np
import torch

from .. import codec
from .._device import flatten_state, to_device_flat, to_host
from ..utils import identity
from .Sharing import Sharing


class STC(Sharing):
    """This class implements STC from https://ieeexplore.ieee.org/document/8889996"""

    def __init__(self, rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                 alpha=1.0, dict_ordered=True, change_transformer=identity, compress=True,
                 compression_package="decentralizepy_amd.compression.EliasFpzipLossy",
                 compression_class="EliasFpzipLossy", float_precision=8):
        super().__init__(rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                         compress, compression_package, compression_class, float_precision)
        self.alpha = alpha
        self.dict_ordered = dict_ordered
        self.change_transformer = change_transformer
        if change_transformer is not identity:
            raise NotImplementedError("STC on the device path supports the identity transformer")
        with torch.no_grad():
            flat = flatten_state(self.model.state_dict())
        self.prev_model = to_device_flat(flat, self.device, self.staging, "local").clone()
        self.residuals = torch.zeros_like(self.prev_model)
        self.model.model_change = torch.zeros_like(self.prev_model)

    # ---- wire format (reference STC.py:96-127) --------------------------------------------------
    def compress_data(self, data):
        result = dict(data)
        if self.compress:
            if "indices" in result:
                result["indices"] = self.compressor.compress(result["indices"])
            if "params" in result:
                result["params"] = self.compressor.compress_float(result["params"])
        return result

    def decompress_data(self, data, device=False):
        data = dict(data)
        if self.compress:
            if "indices" in data:
                data["indices"] = self.compressor.decompress(data["indices"])
            if "params" in data:
                data["params"] = self.compressor.decompress_float(data["params"])
        return data

    def flatten(self, m):
        """reference STC.py:129-143 (host)."""
        with torch.no_grad():
            return torch.cat([v.flatten() for v in m.values()], dim=0)

    def unflatten(self, m):
        """reference STC.py:145-156 (host)."""
        with torch.no_grad():
            result = dict()
            start = 0
            for i, key in enumerate(self.model.state_dict()):
                end = start + self.lens[i]
                result[key] = m[start:end].view(self.shapes[i])
                start = end
        return result

    # ---- helpers --------------------------------------------------------------------------------
    def _k(self):
        return round(self.alpha * self.number_of_params)

    def _flat_model_device(self):
        with torch.no_grad():
            flat = flatten_state(self.model.state_dict())
        return to_device_flat(flat, self.device, self.staging, "local")

    def _message(self, idx, vals):
        m = dict()  # key order of reference STC.py:192-201
        if not self.dict_ordered:
            raise NotImplementedError
        m["alpha"] = self.alpha
        m["indices"] = to_host(idx, self.staging, "idx").astype(np.int32)
        m["params"] = to_host(vals, self.staging, "vals")
        assert len(m["indices"]) == len(m["params"])
        logging.debug("Elements sending: {}".format(len(m["indices"])))
        return self.compress_data(m)

    def _device_sparse(self, m):
        """(idx int32 device, vals fp32 device) of a received, decompressed message."""
        return self._h2d(m["indices"], np.int32, "idx"), self._h2d(m["params"], np.float32, "vals")

    def _encode_change(self):
        """top-k of model_change (STC.py:158-174): (idx, vals) device tensors."""
        return codec.topk_encode(self.model.model_change, self._k(),
                                 vals_src=self.model.model_change, workspace=self.workspace)

    # ---- reference methods ------------------------------------------------------------------------
    def extract_top_gradients(self):
        """reference STC.py:158-174: (values, indices) of the top-k |model_change| (host)."""
        idx, vals = self._encode_change()
        return torch.from_numpy(to_host(vals, self.staging, "vals")), \
            torch.from_numpy(to_host(idx, self.staging, "idx").astype(np.int64))

    def serialized_model(self):
        """reference STC.py:176-205: top-k of model_change as a wire dict."""
        with torch.no_grad():
            idx, vals = self._encode_change()
            return self._message(idx, vals)

    def deserialized_model(self, m, return_flat_tensor=False):
        """reference STC.py:207-241: ``T = zeros(n); T[idx] = params`` (host tensors)."""
        with torch.no_grad():
            m = self.decompress_data(m)
            if not self.dict_ordered:
                raise NotImplementedError
            T = torch.zeros(self.number_of_params)
            index_tensor = torch.tensor(np.asarray(m["indices"]), dtype=torch.long)
            T[index_tensor] = torch.tensor(np.asarray(m["params"]))
            return T if return_flat_tensor else self.unflatten(T)

    def _pre_step(self):
        """reference STC.py:243-254: model_change = flat - prev + residuals; prev = flat."""
        logging.debug("PartialModel _pre_step")
        with torch.no_grad():
            flat = self._flat_model_device()
            change = self.residuals.clone()
            # acc += flat - prev, everywhere (the accumulate-only launch of the encoder, k = 0)
            codec.topk_encode(flat, 0, x0=self.prev_model, acc=change,
                              acc_mode=codec.DPZ_ACC_ACCUMULATE, workspace=self.workspace)
            self.model.model_change = change
            self.prev_model = flat

    def _post_step(self):
        """reference STC.py:256-262"""
        logging.debug("PartialModel _post_step")

    def process_received(self, m=None):
        """reference STC.py:264-303: model = flat + T (flat + 0 without a message)."""
        logging.debug("PartialModel process_received")
        with torch.no_grad():
            flat = self._flat_model_device()
            if m is None:
                idx = torch.empty(0, dtype=torch.int32, device=self.device)
                vals = torch.empty(0, dtype=torch.float32, device=self.device)
            else:
                for key in ("iteration", "degree", "CHANNEL"):
                    if key in m:
                        del m[key]
                idx, vals = self._device_sparse(self.decompress_data(m))
            out = codec.decode_average(flat, [(idx, vals)], add_only=True,
                                       workspace=self.workspace)
            cur_model = torch.from_numpy(to_host(out, self.staging, "result"))
            self.model.load_state_dict(self.unflatten(cur_model))

    def get_data_to_send(self, *args, **kwargs):
        """reference STC.py:305-315, fused: the residual buffer is the encoder's accumulator, so
        residuals += flat - prev, the top-k of |residuals| with values residuals[idx], and
        residuals[idx] = 0 (= model_change - T) are one launch sequence."""
        with torch.no_grad():
            flat = self._flat_model_device()
            k = self._k()
            idx, vals = codec.topk_encode(flat, k, x0=self.prev_model, acc=self.residuals,
                                          acc_mode=codec.DPZ_ACC_ACCUMULATE,
                                          vals_src=self.residuals, workspace=self.workspace)
            self.prev_model = flat
            # model.model_change as the reference leaves it (STC.py:253): the residuals with
            # the sent values put back
            self.model.model_change = codec.replace(self.residuals, idx, vals,
                                                    workspace=self.workspace)
            data = self._message(idx, vals)
            data["iteration"] = self.communication_round
            return data

    def server_broadcast(self, *args, **kwargs):
        """reference STC.py:317-331"""
        with torch.no_grad():
            idx, vals = self._encode_change()
            data = self._message(idx, vals)
            res = self.model.model_change.clone()
            codec.scatter_fill(res, idx, 0.0)  # model_change - T
            self.residuals = res
            self.process_received(data)  # A trick to reuse the code :)
            data["iteration"] = self.communication_round
            return data

    def _averaging_server(self, peer_deques):
        """reference STC.py:333-362: total = sum_i (1/n) T_i from zeros, then
        model_change = residuals + total.  Returns total (host tensor)."""
        with torch.no_grad():
            payloads = []
            weight = 1.0 / len(peer_deques)
            for i, n in enumerate(peer_deques):
                data = peer_deques[n].popleft()
                iteration = data.get("iteration")
                for key in ("iteration", "degree", "CHANNEL"):
                    if key in data:
                        del data[key]
                logging.debug("Averaging model from neighbor {} of iteration {}".format(
                    n, iteration))
                payloads.append(self._device_sparse(self.decompress_data(data)))
            total = codec.decode_average(self.residuals, payloads, [weight] * len(payloads),
                                         None, zero_base=True, workspace=self.workspace)
            # residuals + total (x * 1 is exact; addition commutes)
            self.model.model_change = codec.decode_average(
                self.residuals, [(None, total)], [1.0], 1.0, workspace=self.workspace)
            self.communication_round += 1
        return torch.from_numpy(to_host(total, self.staging, "total"))
