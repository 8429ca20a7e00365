"""raydp-amd: an MI355X-native Spark-on-actors data + training engine with RayDP's API.

Public API parity with ``python/raydp/__init__.py`` of the reference: ``init_spark``,
``stop_spark`` and ``__version__``.
"""
__version__ = "1.7.0.dev0"


def init_spark(*args, **kwargs):
    from raydp_amd.context import init_spark as _init
    return _init(*args, **kwargs)


def stop_spark(cleanup_data=True):
    from raydp_amd.context import stop_spark as _stop
    return _stop(cleanup_data)


__all__ = ["init_spark", "stop_spark", "__version__"]
