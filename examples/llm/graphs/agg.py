from components.frontend import Frontend
from components.processor import Processor
from components.worker import Worker

Frontend.link(Processor).link(Worker)
