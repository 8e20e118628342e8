from components.frontend import Frontend
from components.kv_router import Router
from components.prefill_worker import PrefillWorker
from components.processor import Processor
from components.worker import Worker

Frontend.link(Processor).link(Router).link(Worker).link(PrefillWorker)
