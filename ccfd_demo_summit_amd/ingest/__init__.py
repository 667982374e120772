"""Ingest: brokers (in-process, Kafka wire protocol), producer, message codecs."""
from .broker import BrokerError, Consumer, InProcBroker, Record
from .codec import decode_records, parse_json_batch
from .producer import ProducerConfig, TransactionProducer

__all__ = ["BrokerError", "Consumer", "InProcBroker", "Record", "decode_records", "parse_json_batch",
           "ProducerConfig", "TransactionProducer"]
