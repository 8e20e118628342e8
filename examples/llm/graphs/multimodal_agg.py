"""Aggregated multimodal (LLaVA) graph: Frontend -> Processor -> Worker -> EncodeWorker
(reference examples/multimodal/graphs/agg.py).  The Worker calls the
EncodeWorker for image features when started with `encode-worker: EncodeWorker`."""
from components.encode_worker import EncodeWorker
from components.frontend import Frontend
from components.processor import Processor
from components.worker import Worker

Frontend.link(Processor).link(Worker).link(EncodeWorker)
