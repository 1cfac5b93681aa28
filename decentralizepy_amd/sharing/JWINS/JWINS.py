"""JWINS plugin: Wavelet with a random share fraction per round.

Drop-in for the reference ``decentralizepy.sharing.JWINS.JWINS.JWINS``
(``src/decentralizepy/sharing/JWINS/JWINS.py:12-97``): ``alpha_list`` arrives as a string from
the config and is ``eval``-ed; the process-global ``random`` module is seeded with the node uid and
``alpha = random.choice(alpha_list)`` is drawn every round, so the alpha sequence (and its
interplay with any other use of ``random`` in the process) is the reference's.
"""
import random

from .Wavelet import Wavelet


class JWINS(Wavelet):
    """This class implements the JWINS sharing algorithm."""

    def __init__(self, rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                 alpha_list="[0.1, 0.2, 0.3, 0.4, 1.0]", dict_ordered=True, save_shared=False,
                 metadata_cap=1.0, wavelet="haar", level=4, change_based_selection=True,
                 save_accumulated="", accumulation=False, accumulate_averaging_changes=False,
                 compress=False, compression_package=None, compression_class=None):
        super().__init__(rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                         1.0, dict_ordered, save_shared, metadata_cap, wavelet, level,
                         change_based_selection, save_accumulated, accumulation,
                         accumulate_averaging_changes, compress, compression_package,
                         compression_class)
        self.alpha_list = eval(alpha_list)
        random.seed(self.mapping.get_uid(self.rank, self.machine_id))

    def get_data_to_send(self, degree=None):
        """Perform a sharing step. Implements D-PSGD with alpha randomly chosen.

        As in the reference (JWINS.py:91-97) the degree argument is not forwarded."""
        self.alpha = random.choice(self.alpha_list)
        return super().get_data_to_send()
