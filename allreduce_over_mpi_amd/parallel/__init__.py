from .comm import Communicator, LocalGroup  # noqa: F401
