"""Exception hierarchy (reference: core/raydp-main/src/main/scala/org/apache/spark/
RayDPException.scala:20-23, ``RayDPException extends SparkException``)."""


class RayDPException(RuntimeError):
    """Base of every error raised by the framework's control and data planes."""


class AppMasterError(RayDPException):
    """The application master refused or failed a request (registration, scheduling)."""


class ExecutorLostError(RayDPException):
    """An executor died and its work could not be recovered within the retry budget."""


class ShuffleFetchError(RayDPException):
    """A map output could not be fetched from the shuffle service."""


class CollectiveError(RayDPException):
    """A collective (xGMI one-shot all-reduce / RCCL) failed or timed out."""
