from .comm import Communicator, LocalGroup, file_exchange, store_exchange  # noqa: F401
