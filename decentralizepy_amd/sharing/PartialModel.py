"""PartialModel plugin: top-k magnitude sparsification of the model change, on the MI355X codec.

Drop-in for the reference ``decentralizepy.sharing.PartialModel.PartialModel``
(``src/decentralizepy/sharing/PartialModel.py``): identical constructor keyword arguments
(``alpha, dict_ordered, save_shared, metadata_cap, accumulation, save_accumulated,
change_transformer, accumulate_averaging_changes, compress, compression_package,
compression_class, float_precision``), identical wire payload
``{alpha, indices: int32[k], params: fp32[k], send_partial: True}`` and identical side effects on
the model (``shared_parameters_counter[idx] += 1``, ``accumulated_changes`` accumulate/rewind).

Device state (HBM, fp32): ``init_model`` (x0), ``pre_share_model`` (x), ``accumulated_changes``,
``prev`` and the int32 share counter.  Per round: one H2D of the flat model, one fused HIP top-k
encode (|x - x0| [+acc] -> sampled radix select -> ordered compaction, counter/rewind fused), one
D2H of the (idx, val) payload; on receive one batched replace+fold over all neighbour payloads,
one D2H of the averaged model.

Selection parity: the index set equals the reference's ``torch.topk`` set whenever the k-th key is
unique; at a tie this build takes the lowest indices (torch's CPU choice is implementation-defined,
SURVEY.md §0 item 5).
"""
import json
import logging
import os
from pathlib import Path

import numpy as np
import torch

from .. import codec
from .._device import (DeviceAccumulator, LazyChange, RingCounter, state_to_device,
                       state_version, to_host)
from ..utils import conditional_value, identity
from .Sharing import Sharing


class PartialModel(Sharing):
    """This class implements the vanilla version of partial model sharing."""

    def __init__(self, rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                 alpha=1.0, dict_ordered=True, save_shared=False, metadata_cap=1.0,
                 accumulation=False, save_accumulated="", change_transformer=identity,
                 accumulate_averaging_changes=False, compress=False, compression_package=None,
                 compression_class=None, float_precision=None):
        super().__init__(rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                         compress, compression_package, compression_class, float_precision)
        # reference PartialModel.py:96-145
        self.alpha = alpha
        self.dict_ordered = dict_ordered
        self.save_shared = save_shared
        self.metadata_cap = metadata_cap
        self.accumulation = accumulation
        self.save_accumulated = conditional_value(save_accumulated, "", False)
        self.change_transformer = change_transformer
        self.accumulate_averaging_changes = accumulate_averaging_changes
        if self.save_accumulated:  # reference PartialModel.py:122-131
            self.model_change_path = os.path.join(self.log_dir, "model_change/{}".format(self.rank))
            Path(self.model_change_path).mkdir(parents=True, exist_ok=True)
            self.model_val_path = os.path.join(self.log_dir, "model_val/{}".format(self.rank))
            Path(self.model_val_path).mkdir(parents=True, exist_ok=True)
        self._check_transformer()

        with torch.no_grad():
            self.init_model = state_to_device(self.model.state_dict(), self.device, self.staging,
                                              "local")
        # the fold output can stand in for a re-read of the loaded model only if every state
        # tensor is fp32 (load_state_dict casts other dtypes)
        self._all_fp32 = all(v.dtype == torch.float32 for v in self.model.state_dict().values())
        self._pre_version = None
        self.number_of_params = self.init_model.numel()
        self.transformed_len = self._transformed_len()
        if self.accumulation:
            self.model.accumulated_changes = torch.zeros(self.transformed_len, dtype=torch.float32,
                                                         device=self.device)
            self.prev = self.init_model
        if self.save_shared and not (rank == 0 or rank == 1):
            self.save_shared = False
        if self.save_shared:
            self.folder_path = os.path.join(self.log_dir, "shared_params/{}".format(self.rank))
            Path(self.folder_path).mkdir(parents=True, exist_ok=True)
        # the share counter: each round's payload indices are kept in a device ring and added to
        # the int32 counter when it is read (RingCounter; the encode does no counter update)
        self._counter = torch.zeros(self.transformed_len, dtype=torch.int32, device=self.device)
        self._ring = RingCounter(self._counter)
        self.model.shared_parameters_counter = self._ring
        self.pre_share_model = None
        self.pre_share_model_transformed = None

    # ---- hooks the wavelet subclass overrides --------------------------------------------------
    def _check_transformer(self):
        if self.change_transformer is not identity:
            raise NotImplementedError(
                "PartialModel on the device codec supports the identity change_transformer; "
                "use decentralizepy_amd.sharing.JWINS.Wavelet for the wavelet transform")

    def _transformed_len(self):
        return self.number_of_params

    def _transform_pre_step(self, x):
        """(T(x), T(x - init)) on device; identity: the change is formed inside the encoder."""
        return x, None

    # ---- wire format ------------------------------------------------------------------------------
    def compress_data(self, data, idx_dev=None, val_dev=None):
        """reference PartialModel.py:147-154; a device compressor codes the (already sorted)
        device indices and the device values directly."""
        result = dict(data)
        if self.compress:
            if "indices" in result:
                if idx_dev is not None and hasattr(self.compressor, "compress_device"):
                    result["indices"] = self.compressor.compress_device(idx_dev)
                else:
                    result["indices"] = self.compressor.compress(result["indices"])
            if "params" in result:
                if val_dev is not None and hasattr(self.compressor, "compress_float_device"):
                    result["params"] = self.compressor.compress_float_device(val_dev)
                else:
                    result["params"] = self.compressor.compress_float(result["params"])
        return result

    def decompress_data(self, data, device=False):
        """reference PartialModel.py:156-162; with ``device`` a device compressor decodes the
        indices straight into a device int32 tensor for the fold."""
        if self.compress:
            comp = self.compressor
            if device and getattr(comp, "async_decode", False):
                return self._decompress_async(data)
            if "indices" in data:
                if device and hasattr(comp, "decompress_device"):
                    data["indices"] = comp.decompress_device(data["indices"])
                else:
                    data["indices"] = comp.decompress(data["indices"])
            if "params" in data:
                if device and hasattr(comp, "decompress_float_device"):
                    data["params"] = comp.decompress_float_device(data["params"])
                else:
                    data["params"] = comp.decompress_float(data["params"])
        return data

    def _decompress_async(self, data):
        """The device decode of a received payload with no host synchronisation: the value count
        comes from the float leg's header (or the raw values' length), both legs go up through
        the compressor's pinned ring and decode on the stream, and a malformed leg ORs the
        round's status word, read once after the fold (``_check_received``).  The host copy of
        the next payload's streams then overlaps this one's DMA and decode."""
        comp = self.compressor
        status = self._recv_status_word()
        params = data.get("params")
        if params is not None and hasattr(comp, "decompress_float_device"):
            data["params"] = comp.decompress_float_device(params, status=status)
            count = data["params"].numel()
        else:
            if params is not None:
                data["params"] = comp.decompress_float(params)
                count = int(np.asarray(data["params"]).size)
            else:
                count = 0
        if "indices" not in data:  # a full share (Wavelet.py:174-231's metadata cap)
            return data
        if count < 1:  # nothing to check the index count against: the synchronous decode
            data["indices"] = comp.decompress_device(data["indices"])
        else:
            data["indices"] = comp.decompress_device(data["indices"], count=count, status=status)
        return data

    # ---- encode -----------------------------------------------------------------------------------
    def _acc_mode(self):
        if not self.accumulation:
            return codec.DPZ_ACC_NONE
        return codec.DPZ_ACC_ADD if self.accumulate_averaging_changes else codec.DPZ_ACC_ACCUMULATE

    def _pre_step(self):
        """reference PartialModel.py:305-331: the change (and the accumulation) is fused into the
        encode kernel; here only the flat model moves to the device."""
        logging.debug("PartialModel _pre_step")
        self._fb = None  # a fold base from an earlier round never carries over
        with torch.no_grad():
            sd = self.model.state_dict()
            self.pre_share_model = state_to_device(sd, self.device, self.staging, "local")
            self._pre_version = state_version(sd)
            self.pre_share_model_transformed, self._change_dev = \
                self._transform_pre_step(self.pre_share_model)
            self.model.model_change = self._model_change()

    def _model_change(self):
        """``model.model_change`` as the reference sets it (PartialModel.py:317-331): T(x - init),
        and with accumulation the accumulated change before the rewind (acc + change; fp32
        addition commutes, so it is the same bits as the reference's ``acc += change`` /
        ``change += acc``).  The selection never reads it (the encode fuses the change), so it is
        formed on read (LazyChange) whenever the round leaves its inputs untouched until
        _post_step drops it: no accumulation (x and init_model are never written in place), or
        the deferred-rewind accumulator (DeviceAccumulator: a write through it forms the value
        first).  A plain accumulator is written in place by the encode (rewind, or acc += change
        with DPZ_ACC_ACCUMULATE), so there the value is formed now, before the encode."""
        x, init, change = self.pre_share_model, self.init_model, self._change_dev
        acc = self.model.accumulated_changes if self.accumulation else None
        if acc is None:
            if change is not None:  # T(x - init) was formed for the key (wavelet, FFT)
                return change
            return LazyChange(lambda: self._form_change(x, init, None, None))
        if isinstance(acc, DeviceAccumulator):
            acc_t = acc.settle()
            lz = LazyChange(lambda: self._form_change(x, init, change, acc_t))
            acc.watch(lz)
            return lz
        return self._form_change(x, init, change, acc)

    @staticmethod
    def _form_change(x, init, change, acc):
        """T(x - init) [+ acc] into a new device tensor (DPZ_EW_SUB / DPZ_EW_ADD kernels)."""
        buf = torch.empty_like(change if change is not None else x)
        if change is None:
            codec.elementwise(codec.DPZ_EW_SUB, x, init, out=buf)
            change = buf
        if acc is None:
            return change
        codec.elementwise(codec.DPZ_EW_ADD, acc.view(torch.float32), change.view(torch.float32),
                          out=buf.view(torch.float32))
        return buf

    def _drop_model_change(self):
        """``model.model_change = None`` (reference PartialModel.py:350), and the accumulator no
        longer has to form it before a write."""
        self.model.model_change = None
        acc = getattr(self.model, "accumulated_changes", None)
        if isinstance(acc, DeviceAccumulator):
            acc.unwatch()

    def _ring_slot(self, k):
        """Payload index buffer for this round's encode: a slot of the counter ring (None when
        the counter is kept in another form, e.g. the sliced planes)."""
        ring = getattr(self, "_ring", None)
        return ring.slot(k) if ring is not None and self._counter is not None else None

    def _ring_commit(self, idx):
        """The encode's payload indices are final: they count in shared_parameters_counter."""
        ring = getattr(self, "_ring", None)
        if ring is not None and self._counter is not None:
            ring.commit(idx.numel())

    def _encode(self, k, blocking=True):
        """Top-k encode; returns device (idx int32[k], val fp32[k]).  ``blocking=False`` only
        enqueues it (a sampled-path miss then shows in the workspace's sticky status word and the
        result is not final: the device-time bench's back-to-back rounds, never the plugin's own
        serialized_model, whose payload must be final)."""
        key_src = self._change_dev if self._change_dev is not None else self.pre_share_model
        x0 = None if self._change_dev is not None else self.init_model
        acc = self._acc()
        self._fb = None
        pred = self._predicted_fold() if self._change_dev is None and acc is None else None
        # the payload indices go straight into the counter ring's slot (no counter update here)
        slot = self._ring_slot(k)
        if pred is not None:
            # one neighbour: the encode's filter also writes the fold's no-hit base over x
            # (dpz_topk_encode_foldbase); _averaging then rewrites only the payload's elements
            base = torch.empty_like(self.pre_share_model)
            out = codec.topk_encode(key_src, k, x0=x0, vals_src=self.pre_share_model_transformed,
                                    idx_out=slot, workspace=self.workspace,
                                    fold_base=(base, pred[0], pred[1]), hint=True, keep_x=True,
                                    asynchronous=not blocking)
            self._fb = (base, pred, self.pre_share_model)
            self._ring_commit(out[0])
            return out
        # hint: the previous round's exact threshold as this round's key window (no sample
        # launch); keep_x: _averaging folds over this x right after (Infinity Cache)
        out = codec.topk_encode(key_src, k, x0=x0, acc=acc, acc_mode=self._acc_mode(),
                                vals_src=self.pre_share_model_transformed, idx_out=slot,
                                workspace=self.workspace, hint=True,
                                keep_x=key_src is self.pre_share_model,
                                asynchronous=not blocking)
        self._ring_commit(out[0])
        return out

    def _predicted_fold(self):
        """The Metro-Hastings weights _averaging will use (Sharing.py:156-190), predicted from
        the static graph when the node has exactly ONE neighbour: the only case where writing
        the fold's no-hit base during the encode and patching the payload's elements afterwards
        beats the plain fold (measured on MI355X: one payload 72.4 -> 63.5 us per encode + fold
        at C2, 91.8 -> 80.3 us at 64 MiB; three payloads 94.5 -> 101.1 us at 64 MiB, the patch
        touching most cache lines).  None otherwise."""
        graph = getattr(self, "graph", None)
        if graph is None or not self._all_fp32:
            return None
        try:
            nbrs = list(graph.neighbors(self.uid))
            if len(nbrs) != 1:
                return None
            d = len(graph.neighbors(nbrs[0]))
        except Exception:  # a graph object without the reference interface: plain fold
            return None
        w = 1 / (max(len(nbrs), d) + 1)
        weight_total = 0
        weight_total += w
        return [w], 1 - weight_total

    def _fold_on_base(self, local, payloads, weights, w_self):
        """The round's fold over the base the encode wrote (_encode), when its prediction held:
        same weights, the local term still the encoded model, sparse payloads only."""
        fb, self._fb = getattr(self, "_fb", None), None
        if fb is None:
            return None
        base, (pw, pws), x = fb
        if local is not x or list(weights) != list(pw) or w_self != pws or \
                any(i is None for i, _ in payloads):
            return None
        return codec.decode_average(local, payloads, weights, w_self, out=base,
                                    workspace=self.workspace, base_ready=True)

    def _acc(self):
        """The device accumulator (None without accumulation), any deferred rewind applied."""
        a = self.model.accumulated_changes if self.accumulation else None
        return a.settle() if isinstance(a, DeviceAccumulator) else a

    def _zero_accumulation(self):
        if getattr(self.model, "accumulated_changes", None) is not None:
            self.model.accumulated_changes.zero_()

    def _full_share(self):
        """alpha >= metadata_cap: the whole (transformed) model (reference PartialModel.py:198-203)."""
        self._zero_accumulation()
        return Sharing.serialized_model(self)

    def serialized_model(self):
        """reference PartialModel.py:188-255"""
        if self.alpha >= self.metadata_cap:  # Share fully
            return self._full_share()
        with torch.no_grad():
            k = round(self.alpha * self.transformed_len)
            idx_dev, val_dev = self._encode(k)
            indices = to_host(idx_dev, self.staging, "idx")
            params = to_host(val_dev, self.staging, "val")
            if self.save_shared:
                self._dump_shared(indices)
            if not self.dict_ordered:
                raise NotImplementedError
            m = self._message(indices, params)
            assert len(m["indices"]) == len(m["params"])
            logging.debug("Elements sending: {}".format(len(m["indices"])))
            return self.compress_data(m, idx_dev=idx_dev, val_dev=val_dev)

    def _message(self, indices, params):
        m = dict()  # key order of reference PartialModel.py:235-246
        m["alpha"] = self.alpha
        m["indices"] = indices.astype(np.int32)
        m["params"] = params
        m["send_partial"] = True
        return m

    def _dump_shared(self, indices):
        shared_params = dict()
        shared_params["order"] = list(self.model.state_dict().keys())
        shared_params["shapes"] = {k: list(v.shape) for k, v in self.model.state_dict().items()}
        shared_params[self.communication_round] = indices.tolist()
        with open(os.path.join(self.folder_path,
                               "{}_shared_params.json".format(self.communication_round + 1)),
                  "w") as of:
            json.dump(shared_params, of)

    # ---- decode -----------------------------------------------------------------------------------
    def _device_payload(self, data):
        if "send_partial" not in data:
            return super()._device_payload(data)
        return self._h2d(data["indices"], np.int32, "idx"), self._h2d(data["params"], np.float32,
                                                                        "vals")

    def deserialized_model(self, m):
        """Received dict -> state_dict: ``T = cat(local); T[idx] = params`` on the device
        (reference PartialModel.py:257-303)."""
        if "send_partial" not in m:
            return super().deserialized_model(m)
        with torch.no_grad():
            m = self.decompress_data(m)
            idx, vals = self._device_payload(m)
            local = self._local_flat_device()
            out = codec.replace(local, idx, vals, workspace=self.workspace)
            return self._unflatten(to_host(out, self.staging, "result"))

    def _post_step(self):
        """reference PartialModel.py:333-353; the new model is already on the device (fold output)."""
        logging.debug("PartialModel _post_step")
        # model_change is None after the post-step (reference PartialModel.py:350); dropped first,
        # so the accumulating pass below need not form a lazily kept value nobody can read
        self._drop_model_change()
        with torch.no_grad():
            post = getattr(self, "_post_model_dev", None)
            if post is None or not self._all_fp32:
                post = state_to_device(self.model.state_dict(), self.device, self.staging, "local")
            self._post_model_dev = None
            self.init_model = post
            if self.accumulation:
                if self.accumulate_averaging_changes:
                    self._accumulate_change(self.init_model, self.prev)
                self.prev = self.init_model
        if self.save_accumulated:
            self.save_change()

    def save_vector(self, v, s):
        """reference PartialModel.py:355-383: {order, shapes, tensor} as JSON per round."""
        output_dict = dict()
        output_dict["order"] = list(self.model.state_dict().keys())
        output_dict["shapes"] = {k: list(v1.shape) for k, v1 in self.model.state_dict().items()}
        output_dict["tensor"] = v.tolist()
        with open(os.path.join(s, "{}.json".format(self.communication_round + 1)), "w") as of:
            json.dump(output_dict, of)

    def save_change(self):
        """reference PartialModel.py:385-390.  As in the reference, _post_step has already cleared
        model.model_change, so this raises AttributeError on None (the reference's behaviour
        with save_accumulated set, kept for drop-in fidelity)."""
        self.save_vector(self.model.model_change, self.model_change_path)

    def _accumulate_change(self, new, prev):
        """acc += T(new - prev) (identity: the encoder's accumulate-only kernel)."""
        codec.topk_encode(new, 0, x0=prev, acc=self.model.accumulated_changes,
                          acc_mode=codec.DPZ_ACC_ACCUMULATE, workspace=self.workspace)

    def _local_flat_device(self):
        """The fold's local term: the pre-share copy if the model was not touched since
        _pre_step (torch version counters), else a fresh H2D of the current model."""
        if self.pre_share_model is not None and self._pre_version == state_version(
                self.model.state_dict()):
            return self.pre_share_model
        return super()._local_flat_device()

    def _load_flat(self, out_dev):
        super()._load_flat(out_dev)
        self._post_model_dev = out_dev
