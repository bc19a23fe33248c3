"""warpcore_amd -- MI355X (gfx950) implementation of warpcore's per-packet
Internet / UDP checksum hot path (lib/src/in_cksum.c in the reference).

Product: ``libwccksum.so`` (HIP kernels + C ABI, ``include/warpcore_gpu``).
This package is the Python host mirror of that C ABI plus the synthetic
packet generators and the multi-GPU shard driver used by bench.py.
"""
from .cksum import (KIND_IP, KIND_PAYLOAD, SclkProbe, WcError, cksum_host, cksum_host_multi,
                    cksum_ip_udp_host, server_pause, server_paused, server_resume,
                    server_stats,
                    cksum_ip_udp_ragged, cksum_ragged_multi, gather_results_multi,
                    gpu_init_multi, shard_range,
                    cksum_ip_udp_strided, cksum_ragged, cksum_strided, gpu_init, host_register, host_unregister,
                    ip_cksum, payload_cksum, plan_strided, reload_config, synth_fill,
                    verify_ragged, verify_strided, version, shard_devices,
                    rx_verdict_ragged, rx_verdict_host, RX_NAMES, RX_DROPS,
                    RX_OK, RX_OK_NO_CKSUM, RX_BAD_IP_CKSUM, RX_BAD_UDP_CKSUM, RX_SHORT,
                    RX_FRAGMENT, RX_BAD_VERSION, RX_NOT_UDP, RX_NOT_IP, RX_TRUNCATED)

__all__ = [
    "KIND_IP", "KIND_PAYLOAD", "SclkProbe", "WcError", "cksum_host", "cksum_host_multi",
    "cksum_ip_udp_host", "server_pause", "server_paused", "server_resume", "server_stats",
    "cksum_ip_udp_ragged", "cksum_ragged_multi", "gather_results_multi", "gpu_init_multi",
    "shard_range",
    "cksum_ip_udp_strided", "cksum_ragged",
    "cksum_strided", "gpu_init", "host_register", "host_unregister", "ip_cksum",
    "payload_cksum", "plan_strided", "reload_config", "synth_fill", "verify_ragged",
    "verify_strided", "version", "shard_devices", "rx_verdict_ragged", "rx_verdict_host",
    "RX_NAMES", "RX_DROPS", "RX_OK", "RX_OK_NO_CKSUM", "RX_BAD_IP_CKSUM", "RX_BAD_UDP_CKSUM",
    "RX_SHORT", "RX_FRAGMENT", "RX_BAD_VERSION", "RX_NOT_UDP", "RX_NOT_IP", "RX_TRUNCATED",
]
