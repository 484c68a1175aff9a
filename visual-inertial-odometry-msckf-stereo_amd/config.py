"""Filter configuration for the MI355X MSCKF update path.

Mirrors the filter-relevant fields of the reference ConfigEuRoC /
OptimizationConfigEuRoC (MSCKF/config.py:5-124).  Front-end fields (FAST,
KLT, grid) are out of scope and not carried.  Values are the reference's
defaults.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# chi2.ppf(0.05, dof) for dof = 1..99, exactly as the reference builds it
# (MSCKF/msckf.py:121-123 -- note the 5 % LOWER quantile, quirk Q6).  Generated
# once with scipy 1.15.3 and frozen here so that no scipy is needed at run time.
CHI2_05 = (
    0.003932140000019522, 0.10258658877510106, 0.35184631774927144,
    0.7107230213973239, 1.1454762260617692, 1.6353828943279067,
    2.167349909298057, 2.732636793499662, 3.325112843066815,
    3.9402991361190605, 4.574813079322224, 5.226029488392639,
    5.8918643377098485, 6.57063138378934, 7.2609439276700325,
    7.9616455723785515, 8.671760204670077, 9.390455080688984,
    10.117013063859044, 10.85081139418259, 11.591305208820733,
    12.338014578790643, 13.090514188172804, 13.848425027170224,
    14.61140763948331, 15.379156583261723, 16.151395849664098,
    16.927875044422496, 17.70836618282458, 18.49266098195347,
    19.280568559129293, 20.071913464548288, 20.86653399071479,
    21.664280712551975, 22.465015220882684, 23.268609018893773,
    24.07494255667991, 24.883904383335626, 25.695390399574777,
    26.50930319669311, 27.32555146999419, 28.144049496682623,
    28.964716669775694, 29.787477080861958, 30.612259145595477,
    31.43899526669704, 32.26762152997339, 33.09807742948629,
    33.93030561852784, 34.76425168350175, 35.5998639381883,
    36.437093236191636, 37.275892799644296, 38.1162180624794,
    38.95802652678509, 39.80127763093126, 40.64593262831063,
    41.491954475668955, 42.33930773011346, 43.187958453989765,
    44.03787412690472, 44.88902356425022, 45.741376841650336,
    46.594905224813964, 47.44958110432793, 48.30537793497176,
    49.16227017917681, 50.020233254289266, 50.879243483328636,
    51.73927804896291, 52.60031495044724, 53.462332963296205,
    54.325311601480685, 55.1892310819587, 56.05407229136661,
    56.91981675471199, 57.78644660592318, 58.65394456012262,
    59.52229388750226, 60.391478388689464, 61.261482371500676,
    62.13229062898852, 63.003888418695496, 63.87626144303417,
    64.74939583071999, 65.62327811918864, 66.49789523793463,
    67.37323449271317, 68.24928355055083, 69.12603042551552,
    70.00346346519876, 70.88157133786743, 71.76034302024499,
    72.63976778588469, 73.5198351941001, 74.40053507942093,
    75.28185754154367, 76.16379293574907, 77.04633186376029,
)


def chi2_threshold(dof: int) -> float:
    """Reference chi_squared_test_table[dof] (msckf.py:611).  The table has
    keys 1..99; any other dof raises KeyError like the reference dict."""
    if dof < 1 or dof > 99:
        raise KeyError(dof)
    return CHI2_05[dof - 1]


@dataclass
class OptimizationConfig:
    """Reference OptimizationConfigEuRoC (config.py:5-15)."""
    translation_threshold: float = -1.0
    huber_epsilon: float = 0.01
    estimation_precision: float = 5e-7
    initial_damping: float = 1e-3
    outer_loop_max_iteration: int = 5
    inner_loop_max_iteration: int = 5


def _default_T_imu_cam0():
    return np.array([
        [0.014865542981794, 0.999557249008346, -0.025774436697440, 0.065222909535531],
        [-0.999880929698575, 0.014967213324719, 0.003756188357967, -0.020706385492719],
        [0.004140296794224, 0.025715529947966, 0.999660727177902, -0.008054602460030],
        [0, 0, 0, 1.000000000000000]])


def _default_T_cn_cnm1():
    return np.array([
        [0.999997256477881, 0.002312067192424, 0.000376008102415, -0.110073808127187],
        [-0.002317135723281, 0.999898048506644, 0.014089835846648, 0.000399121547014],
        [-0.000343393120525, -0.014090668452714, 0.999900662637729, -0.000853702503357],
        [0, 0, 0, 1.000000000000000]])


@dataclass
class FilterConfig:
    """Filter fields of the reference ConfigEuRoC (config.py:17-124)."""
    optimization: OptimizationConfig = field(default_factory=OptimizationConfig)
    gravity: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -9.81]))
    max_cam_state_size: int = 20
    position_std_threshold: float = 8.0
    gyro_noise: float = 0.005 ** 2
    acc_noise: float = 0.05 ** 2
    gyro_bias_noise: float = 0.001 ** 2
    acc_bias_noise: float = 0.01 ** 2
    observation_noise: float = 0.035 ** 2
    velocity: np.ndarray = field(default_factory=lambda: np.zeros(3))
    velocity_cov: float = 0.25
    gyro_bias_cov: float = 0.01
    acc_bias_cov: float = 0.01
    extrinsic_rotation_cov: float = 3.0462e-4
    extrinsic_translation_cov: float = 2.5e-5
    T_imu_cam0: np.ndarray = field(default_factory=_default_T_imu_cam0)
    T_cn_cnm1: np.ndarray = field(default_factory=_default_T_cn_cnm1)
    T_imu_body: np.ndarray = field(default_factory=lambda: np.eye(4))

    @classmethod
    def from_reference(cls, ref_cfg) -> "FilterConfig":
        """Build from a reference-style config object (the attribute names the
        reference uses, config.py:9-124), so a caller holding a ConfigEuRoC
        can pass it straight through."""
        g = lambda n: getattr(ref_cfg, "_vio_%s__" % n)
        oc = g("optimization_config")
        go = lambda n: getattr(oc, "_vio_%s__" % n)
        return cls(
            optimization=OptimizationConfig(
                go("translation_threshold"), go("huber_epsilon"),
                go("estimation_precision"), go("initial_damping"),
                go("outer_loop_max_iteration"), go("inner_loop_max_iteration")),
            gravity=np.array(g("gravity"), float),
            max_cam_state_size=g("max_cam_state_size"),
            position_std_threshold=g("position_std_threshold"),
            gyro_noise=g("gyro_noise"), acc_noise=g("acc_noise"),
            gyro_bias_noise=g("gyro_bias_noise"), acc_bias_noise=g("acc_bias_noise"),
            observation_noise=g("observation_noise"),
            velocity=np.array(g("velocity"), float),
            velocity_cov=g("velocity_cov"), gyro_bias_cov=g("gyro_bias_cov"),
            acc_bias_cov=g("acc_bias_cov"),
            extrinsic_rotation_cov=g("extrinsic_rotation_cov"),
            extrinsic_translation_cov=g("extrinsic_translation_cov"),
            T_imu_cam0=np.array(g("T_imu_cam0"), float),
            T_cn_cnm1=np.array(g("T_cn_cnm1"), float),
            T_imu_body=np.array(g("T_imu_body"), float))
