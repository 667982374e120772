"""Env-var config keys and their reference defaults (SURVEY.md §2.3 "Env-var config keys").

Loading order used by :func:`ccfd_demo_summit_amd.config.load_config`:
defaults (the reference values below) -> YAML file -> the SAME env var names -> CLI.
"""

# key: (default, type, where the reference sets it)
REFERENCE_ENV = {
    "BROKER_URL": ("odh-message-bus-kafka-brokers:9092", str, "router.yaml:55-56; ccd-service.yaml:55-56"),
    "KAFKA_TOPIC": ("odh-demo", str, "router.yaml:61-62"),
    "CUSTOMER_NOTIFICATION_TOPIC": ("ccd-customer-outgoing", str, "router.yaml:57-58; ccd-service.yaml:57-58"),
    "CUSTOMER_RESPONSE_TOPIC": ("ccd-customer-response", str, "router.yaml:59-60"),
    "KIE_SERVER_URL": ("http://ccd-service:8090", str, "router.yaml:63-64"),
    "SELDON_URL": ("http://modelfull-modelfull:8000", str, "router.yaml:67-68"),
    "SELDON_ENDPOINT": ("api/v0.1/predictions", str, "router.yaml:65-66 (KIE default 'predict', README.md:379)"),
    "SELDON_TOKEN": (None, str, "README.md:372-377,447-452"),
    "SELDON_TIMEOUT": (5000, int, "README.md:386-393 (ms)"),
    "SELDON_POOL_SIZE": (5, int, "README.md:386-393"),
    "CONFIDENCE_THRESHOLD": (1.0, float, "README.md:395-402"),
    "FRAUD_THRESHOLD": (0.5, float, "router.yaml:69-70"),
    "NEXUS_URL": ("http://nexus:8081", str, "ccd-service.yaml:59-60 (unused: processes are code)"),
    # producer (ProducerDeployment.yaml:77-97)
    "topic": ("odh-demo", str, "ProducerDeployment.yaml:88-89"),
    "s3endpoint": (None, str, "ProducerDeployment.yaml:90-91"),
    "s3bucket": ("ccdata", str, "ProducerDeployment.yaml:92-93"),
    "filename": ("OPEN/uploaded/creditcard.csv", str, "ProducerDeployment.yaml:94-95"),
    "bootstrap": ("odh-message-bus-kafka-bootstrap:9092", str, "ProducerDeployment.yaml:96-97"),
    "ACCESS_KEY_ID": (None, str, "ProducerDeployment.yaml:78-82 (secret keysecret)"),
    "SECRET_ACCESS_KEY": (None, str, "ProducerDeployment.yaml:83-87"),
}

# The KIE prediction service uses a different SELDON_URL default than the router
# (ccd-service.yaml:61-62 vs router.yaml:67-68).
KIE_SELDON_URL_DEFAULT = "ccfd-seldon-model:5000"
KIE_SELDON_ENDPOINT_DEFAULT = "predict"
