from .comm import Communicator, LocalGroup, file_exchange, store_exchange  # noqa: F401
from .hierarchical import HierarchicalCommunicator  # noqa: F401
from .graphs import CapturedAllReduce  # noqa: F401
