"""Choco-SGD sharing plugin on the MI355X codec.

Drop-in for the reference ``decentralizepy.sharing.Choco.Choco`` (``src/decentralizepy/sharing/
Choco.py``): same constructor (``step_size, alpha, compress, compression_package,
compression_class, float_precision``), same wire dicts (``{params, indices:int64, send_partial}``
+ ``degree``/``iteration``), same update.

Device path (all HIP kernels, fp32, bit-exact with the reference's operation order):
  _pre_step   d = x - x_hat (elementwise); T = the k-th largest |d| with EVERY tie kept and the
              nonzero filter (``dpz_topk_threshold``: the exact radix path, which also resolves T
              for k = 0 as 0 = no sparsification); q = d with |d| < T zeroed (``dpz_mask_below_
              threshold``) — reference Choco.py:117-161, 362-370
  _averaging  x_hat += q; s += w_i T_i over the neighbours (zero-based sparse payloads, one
              batched fold continuing s in place) + (1 - sum w) q; x += step_size (s - x_hat)
              (Choco.py:412-447)
State kept in HBM across rounds: x_hat (model_hat), s, q (N fp32 each).
"""
import logging
from collections import OrderedDict

import numpy as np
import torch

from .. import codec
from .._device import flatten_state, to_device_flat, to_host
from .Sharing import Sharing


class Choco(Sharing):
    """API defining who to share with and what, and what to do on receiving"""

    def __init__(self, rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                 step_size, alpha, compress=False, compression_package=None,
                 compression_class=None, float_precision=None):
        super().__init__(rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                         compress, compression_package, compression_class, float_precision)
        self.step_size = step_size
        self.alpha = alpha
        logging.debug("type(step_size): %s, value: %s", str(type(self.step_size)),
                      str(self.step_size))
        logging.debug("type(alpha): %s, value: %s", str(type(self.alpha)), str(self.alpha))
        n = self.number_of_params
        self._x_hat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._s = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._q = None
        self._q_idx = self._q_vals = None

    # ---- reference attributes as host state dicts (inspection; the device copies are used) ----
    def _as_state_dict(self, flat_dev):
        flat = torch.from_numpy(to_host(flat_dev, self.staging, "inspect"))
        out, start = OrderedDict(), 0
        for i, key in enumerate(self.model.state_dict()):
            out[key] = flat[start:start + self.lens[i]].view(self.shapes[i])
            start += self.lens[i]
        return out

    @property
    def model_hat(self):
        return self._as_state_dict(self._x_hat)

    @property
    def s(self):
        return self._as_state_dict(self._s)

    @property
    def my_q(self):
        return None if self._q is None else self._as_state_dict(self._q)

    # ---- wire format (reference Choco.py:334-352) ------------------------------------------------
    def compress_data(self, data):
        result = dict(data)
        if self.compress:
            if "indices" in result:
                result["indices"] = self.compressor.compress(result["indices"])
            if "params" in result:
                result["params"] = self.compressor.compress_float(result["params"])
        return result

    def decompress_data(self, data, device=False):
        if self.compress:
            if "indices" in data:
                data["indices"] = self.compressor.decompress(data["indices"])
            if "params" in data:
                data["params"] = self.compressor.decompress_float(data["params"])
        return data

    def _flat_model_device(self):
        with torch.no_grad():
            flat = flatten_state(self.model.state_dict())
        return to_device_flat(flat, self.device, self.staging, "local")

    # ---- round hooks ------------------------------------------------------------------------------
    def _pre_step(self):
        """reference Choco.py:362-370: my_q = topk_sparsification(model - model_hat, alpha)."""
        with torch.no_grad():
            x = self._flat_model_device()
            d = codec.elementwise(codec.DPZ_EW_SUB, x, self._x_hat)
            k = round(self.alpha * d.numel())
            self._q_idx, self._q_vals = codec.topk_threshold(d, k, workspace=self.workspace)
            self._q = codec.mask_below_threshold(d, self.workspace)  # in place: d -> q

    def serialized_model(self):
        """reference Choco.py:372-388: the nonzero entries of my_q."""
        data = dict()
        data["params"] = to_host(self._q_vals, self.staging, "vals")
        data["indices"] = to_host(self._q_idx, self.staging, "idx").astype(np.int64)
        data["send_partial"] = True
        return self.compress_data(data)

    def deserialized_model(self, m):
        """reference Choco.py:390-410 (host state dict of the sparse message)."""
        if "send_partial" not in m:
            return super().deserialized_model(m)
        with torch.no_grad():
            m = self.decompress_data(m)
            indices = torch.tensor(np.asarray(m["indices"]), dtype=torch.long)
            values = torch.tensor(np.asarray(m["params"]))
            T = torch.zeros(self.number_of_params)
            if len(indices):
                T[indices] = values
            out, start = OrderedDict(), 0
            for i, key in enumerate(self.model.state_dict()):
                out[key] = T[start:start + self.lens[i]].reshape(self.shapes[i])
                start += self.lens[i]
            return out

    def _device_message(self, data):
        data = self.decompress_data(data)
        vals = self._h2d(data["params"], np.float32, "vals")
        if "send_partial" not in data:  # a full model (Sharing.deserialized_model)
            return None, vals
        return self._h2d(data["indices"], np.int32, "idx"), vals

    def _averaging(self, peer_deques):
        """reference Choco.py:412-447"""
        with torch.no_grad():
            # x_hat = q_self + x_hat (1.0 * q is exact)
            codec.elementwise(codec.DPZ_EW_ADD, self._x_hat, self._q, out=self._x_hat)
            payloads, weights = [], []
            weight_total = 0
            for i, n in enumerate(peer_deques):
                data = peer_deques[n].popleft()
                degree, iteration = data["degree"], data["iteration"]
                del data["degree"]
                del data["iteration"]
                del data["CHANNEL"]
                logging.debug("Averaging model from neighbor {} of iteration {}".format(
                    n, iteration))
                payloads.append(self._device_message(data))
                weight = 1 / (max(len(peer_deques), degree) + 1)  # Metro-Hastings
                weight_total += weight
                weights.append(weight)
            # s += w_i T_i (payload order), then s += (1 - sum w) q: one fold continuing s
            codec.decode_average(self._q, payloads, weights, 1 - weight_total, out=self._s,
                                 zero_base=True, accumulate=True, workspace=self.workspace)
            x = self._flat_model_device()
            codec.elementwise(codec.DPZ_EW_CHOCO, x, self._s, self._x_hat, self.step_size, out=x)
            flat = torch.from_numpy(to_host(x, self.staging, "result"))
            total = OrderedDict()
            start = 0
            for i, key in enumerate(self.model.state_dict()):
                total[key] = flat[start:start + self.lens[i]].view(self.shapes[i])
                start += self.lens[i]
        self.model.load_state_dict(total)
        self._post_step()
        self.communication_round += 1

    def _averaging_server(self, peer_deques):
        """reference Choco.py:449-455"""
        raise NotImplementedError()
