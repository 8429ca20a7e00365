"""Version constants (reference: ``python/raydp/versions.py``).

The reference picks a log4j flavour from the installed PySpark version because its Spark
master and executors are JVM processes. Our master/executors are native processes that log
through ``raydp_amd.utils.logging`` (no JVM), so the constants are kept only for API parity
with code that imports them; ``SPARK_COMPAT_VERSION`` is the Spark API level our DataFrame
engine mirrors.
"""
__all__ = ["RAYDP_VERSION", "SPARK_COMPAT_VERSION", "SPARK_LOG4J_VERSION",
           "SPARK_LOG4J_CONFIG_FILE_NAME_KEY", "SPARK_LOG4J_CONFIG_FILE_NAME_DEFAULT",
           "RAY_LOG4J_VERSION", "RAY_LOG4J_CONFIG_FILE_NAME_KEY", "RAY_LOG4J_CONFIG_FILE_NAME_DEFAULT"]

RAYDP_VERSION = "1.7.0.dev0"
SPARK_COMPAT_VERSION = "3.5"
SPARK_LOG4J_VERSION = "log4j2"
SPARK_LOG4J_CONFIG_FILE_NAME_KEY = "log4j2.configurationFile"
SPARK_LOG4J_CONFIG_FILE_NAME_DEFAULT = "log4j2-default.properties"
RAY_LOG4J_VERSION = "log4j2"
RAY_LOG4J_CONFIG_FILE_NAME_KEY = "log4j2.configurationFile"
RAY_LOG4J_CONFIG_FILE_NAME_DEFAULT = "log4j2.xml"
