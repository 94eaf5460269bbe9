"""The CAM-TMP temperature schedule of the training loader (dlib/cams/decay_temp.py:20-98).

``DecayTemp`` owns the knobs of the temporal CAM max the trainer builds its seeds from
(datasets/wsol_loader.py:571-601):

* ``sl_tc_knn_t`` — the heating temperature of ``re_normalize_cam`` (:630-635).  With
  ``sl_tc_knn_epoch_switch_uniform`` = -1 it is constant; otherwise it decays linearly
  from ``sl_tc_knn_t`` to ``sl_tc_min_t``, reaching it at epoch
  ``sl_tc_knn_epoch_switch_uniform`` (decay_temp.py:36-55);
* ``sl_tc_seed_tech`` — the seeder's sampling: the configured technique, switched to
  ``seed_uniform`` from epoch ``sl_tc_knn_epoch_switch_uniform`` on (:65-73; the trainer
  applies it in ``on_epoch_start``, learning/train_wsol.py:955-962).

:func:`heat_t` is the loader's gate: the CAMs are heated only when ``sl_tc_knn > 0``
(``_is_tmp``, wsol_loader.py:571, 594) — a single-frame "window" is never heated.
"""
from __future__ import annotations

from .parallel import TIME_DEPENDENCY
from .seeding import SEED_TECHS, SEED_UNIFORM

__all__ = ["DecayTemp", "heat_t"]


def heat_t(sl_tc_knn: int, sl_tc_knn_t: float) -> float:
    """The temperature the temporal max applies: wsol_loader.py:571 ``_is_tmp =
    sl_tc_knn > 0`` and :594 ``if _is_tmp and sl_tc_knn_t > 0`` (0 = no heating)."""
    return float(sl_tc_knn_t) if (sl_tc_knn > 0 and sl_tc_knn_t > 0) else 0.0


class DecayTemp:
    """decay_temp.py:20-98."""

    def __init__(self, sl_tc_knn_t: float, sl_tc_min_t: float, sl_tc_knn: int,
                 sl_tc_knn_mode: str, sl_tc_knn_epoch_switch_uniform: int,
                 sl_tc_seed_tech: str):
        self._sl_tc_knn_mode = sl_tc_knn_mode
        self._sl_tc_knn = sl_tc_knn
        self._sl_tc_knn_t = sl_tc_knn_t
        self._sl_tc_min_t = sl_tc_min_t
        self._sl_tc_knn_epoch_switch_uniform = sl_tc_knn_epoch_switch_uniform
        self._sl_tc_seed_tech = sl_tc_seed_tech
        assert self._sl_tc_knn_t >= self._sl_tc_min_t
        assert sl_tc_knn_mode in TIME_DEPENDENCY
        assert sl_tc_seed_tech in SEED_TECHS
        self.decay = 0.0
        self.decayable = sl_tc_knn_epoch_switch_uniform != -1
        if self.decayable and sl_tc_knn_epoch_switch_uniform > 0:
            self.decay = (self._sl_tc_knn_t - self._sl_tc_min_t) / float(
                sl_tc_knn_epoch_switch_uniform)
        self.epoch = 0

    @property
    def sl_tc_knn_t(self) -> float:
        if not self.decayable:
            return self._sl_tc_knn_t
        return max(self._sl_tc_min_t, self._sl_tc_knn_t - self.epoch * self.decay)

    @property
    def sl_tc_knn_mode(self) -> str:
        return self._sl_tc_knn_mode

    @property
    def sl_tc_knn(self) -> int:
        return self._sl_tc_knn

    @property
    def sl_tc_seed_tech(self) -> str:
        if self.decayable and self.epoch >= self._sl_tc_knn_epoch_switch_uniform:
            return SEED_UNIFORM
        return self._sl_tc_seed_tech

    @property
    def heat_t(self) -> float:
        """The temperature the loader applies this epoch (see :func:`heat_t`)."""
        return heat_t(self.sl_tc_knn, self.sl_tc_knn_t)

    def set_epoch(self, epoch: int) -> None:
        assert isinstance(epoch, int), type(epoch)
        assert epoch >= 0, epoch
        self.epoch = epoch

    def get_current_status(self) -> str:
        return (f"epoch={self.epoch},sl_tc_knn_t={self.sl_tc_knn_t},"
                f"sl_tc_knn_mode={self.sl_tc_knn_mode}, sl_tc_knn={self.sl_tc_knn}, "
                f"sl_tc_seed_tech={self.sl_tc_seed_tech}.")

    def __str__(self):
        return (f"{self.__class__.__name__}(): Decay_tmp. "
                f"_sl_tc_knn_mode = {self._sl_tc_knn_mode}. _sl_tc_knn = {self._sl_tc_knn}. "
                f"_sl_tc_knn_t = {self._sl_tc_knn_t}. _sl_tc_min_t = {self._sl_tc_min_t}. "
                f"_sl_tc_knn_epoch_switch_uniform = {self._sl_tc_knn_epoch_switch_uniform}. "
                f"_sl_tc_seed_tech = {self._sl_tc_seed_tech}.")
