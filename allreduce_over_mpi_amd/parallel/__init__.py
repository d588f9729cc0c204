from .comm import Communicator, LocalGroup, store_exchange  # noqa: F401
