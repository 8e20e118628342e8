from components.frontend import Frontend
from components.prefill_worker import PrefillWorker
from components.processor import Processor
from components.worker import Worker

Frontend.link(Processor).link(Worker).link(PrefillWorker)
